/*
 * mac.h — MAC auto-discovery (the reference's get_src_mac_address / get_gw_mac,
 * src/sequence.c:111-130; PB-Common utils, un-vendored).  See mac.c.
 */
#pragma once

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int pb_get_src_mac_address(const char *dev, uint8_t mac[6]);
int pb_get_gw_mac(uint8_t mac[6]);

/* the same on explicit files (tests, containers with another /proc) */
int pb_get_src_mac_from(const char *addr_path, uint8_t mac[6]);
int pb_get_gw_mac_from(const char *route_path, const char *arp_path, uint8_t mac[6]);

#ifdef __cplusplus
}
#endif
