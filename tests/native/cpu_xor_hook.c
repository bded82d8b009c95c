/* TEST DOUBLE: a plain CPU fold with the bcp_xor_hook_fn signature, so the
 * host protocol layer (process_task over loopback ranks) can be exercised on
 * machines without a GPU.  Not part of the product; compiled by tests. */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

int test_cpu_xor(uint8_t *dst, size_t nbytes, const uint8_t *data, size_t pitch, int nsrc, void *ctx)
{
    (void)ctx;
    memcpy(dst, data, nbytes);
    for (int k = 1; k < nsrc; k++) {
        const uint8_t *s = data + (size_t)k * pitch;
        for (size_t i = 0; i < nbytes; i++)
            dst[i] ^= s[i];
    }
    return 0;
}
