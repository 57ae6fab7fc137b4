/*
 * config_json.h — the reference's JSON config (README.md:170-578) read into
 * pb_config_t, in place of PB-Common's parse_config() (src/main.c:94).  See
 * config_json.c.
 */
#pragma once

#include <stddef.h>

#include "../../include/pb_config.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fills cfg->interface and cfg->seq[0 .. *seq_cnt) over the defaults already
 * there (clear_sequence).  0 on success; -errno (file) or -EINVAL (syntax),
 * with a message on stderr when log != 0. */
int pb_parse_config(const char *path, pb_config_t *cfg, int *seq_cnt, int log);
int pb_parse_config_text(const char *text, size_t len, pb_config_t *cfg, int *seq_cnt, const char **err);
/* frees the strings every parse so far left in the configs */
void pb_config_free(void);

#ifdef __cplusplus
}
#endif
