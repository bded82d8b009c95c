/* bcp_host.h -- internal to the C host layer of libbcp.so (not the ABI; the
 * bcpi_ prefix keeps these out of the export map). */
#pragma once

#include "bcp_task.h"

/* Failure injection (bcp_task_inject_failure): 1 if this pass through
 * `site` must fail. */
int bcpi_inject_hit(int site);
/* Non-zero once this library initialised a HIP runtime that found a device
 * (bcp_engine.hip): a forked child could not use it. */
int bcpi_hip_touched(void);

/* The P-role settings of this process (fold mode, fold service width, test
 * hook, window padding): a rank pool (bcp_runner.c) hands the caller's
 * settings to its rank processes with every run. */
typedef struct {
    int fold_mode, fold_inflight, explicit_pad;
    bcp_xor_hook_fn hook;
    void *hook_ctx;
} bcpi_settings;
void bcpi_settings_get(bcpi_settings *s);
int bcpi_settings_apply(const bcpi_settings *s);
