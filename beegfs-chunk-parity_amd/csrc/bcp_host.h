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
