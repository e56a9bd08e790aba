/*
 * enc_frame_hooks.c — the frame-level entry points of libsvtgpu inside the reference encoder (test infrastructure).
 * Placeholder of the interposed frame-level calls: the hooks are off and every call stays the encoder's own.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static int      g_on;
static uint64_t g_calls;

void enc_frame_hooks_enable(int on) {
    if (on) {
        fprintf(stderr, "enc_drop_in: frame-level hooks not built\n");
        exit(5);
    }
    g_on = on;
}
uint64_t enc_frame_hook_calls(void) { return g_calls; }
