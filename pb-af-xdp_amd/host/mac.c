/*
 * mac.c — MAC auto-discovery for sequences without smac / dmac.
 *
 * The reference resolves a zero source MAC with get_src_mac_address(device)
 * and a zero destination MAC with get_gw_mac() before its packet loop
 * (src/sequence.c:111-130).  Both live in the un-vendored PB-Common utils; this
 * is the build's own restatement on the kernel's text interfaces:
 *   source       /sys/class/net/<device>/address
 *   destination  the default route's gateway (/proc/net/route: destination 0,
 *                RTF_GATEWAY) looked up in the neighbour table (/proc/net/arp)
 * Return 0 on success, a negative errno otherwise (mac left unchanged).
 */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "mac.h"

#define PB_RTF_GATEWAY 0x2 /* linux/route.h */

static int parse_mac_text(const char *s, uint8_t mac[6])
{
    unsigned int b[6];
    if (sscanf(s, "%x:%x:%x:%x:%x:%x", &b[0], &b[1], &b[2], &b[3], &b[4], &b[5]) != 6)
        return -EINVAL;
    for (int i = 0; i < 6; ++i)
    {
        if (b[i] > 0xFF)
            return -EINVAL;
        mac[i] = (uint8_t)b[i];
    }
    return 0;
}

int pb_get_src_mac_from(const char *addr_path, uint8_t mac[6])
{
    FILE *f = fopen(addr_path, "r");
    if (f == NULL)
        return -errno;
    char line[64] = {0};
    const int ok = fgets(line, sizeof line, f) != NULL;
    fclose(f);
    return ok ? parse_mac_text(line, mac) : -EIO;
}

int pb_get_src_mac_address(const char *dev, uint8_t mac[6])
{
    if (dev == NULL || *dev == '\0' || strchr(dev, '/') != NULL || strlen(dev) > 64)
        return -EINVAL;
    char path[128];
    snprintf(path, sizeof path, "/sys/class/net/%s/address", dev);
    return pb_get_src_mac_from(path, mac);
}

int pb_get_gw_mac_from(const char *route_path, const char *arp_path, uint8_t mac[6])
{
    FILE *f = fopen(route_path, "r");
    if (f == NULL)
        return -errno;
    char line[512];
    unsigned int gw = 0;
    int found = 0;
    if (fgets(line, sizeof line, f) == NULL) /* header */
    {
        fclose(f);
        return -EIO;
    }
    while (!found && fgets(line, sizeof line, f) != NULL)
    {
        char iface[64];
        unsigned int dst, gate, flags;
        if (sscanf(line, "%63s %x %x %x", iface, &dst, &gate, &flags) == 4 && dst == 0 && (flags & PB_RTF_GATEWAY))
        {
            gw = gate; /* network order as read from memory: first octet in the low byte */
            found = 1;
        }
    }
    fclose(f);
    if (!found)
        return -ENOENT;
    char ip[32];
    snprintf(ip, sizeof ip, "%u.%u.%u.%u", gw & 0xFF, (gw >> 8) & 0xFF, (gw >> 16) & 0xFF, gw >> 24);

    f = fopen(arp_path, "r");
    if (f == NULL)
        return -errno;
    int rc = -ENOENT;
    if (fgets(line, sizeof line, f) != NULL) /* header */
    {
        while (fgets(line, sizeof line, f) != NULL)
        {
            char a_ip[64], hw[64];
            unsigned int type, flags;
            if (sscanf(line, "%63s %x %x %63s", a_ip, &type, &flags, hw) == 4 && strcmp(a_ip, ip) == 0)
            {
                rc = parse_mac_text(hw, mac);
                break;
            }
        }
    }
    fclose(f);
    return rc;
}

int pb_get_gw_mac(uint8_t mac[6])
{
    return pb_get_gw_mac_from("/proc/net/route", "/proc/net/arp", mac);
}
