/*
 * rtcd_install.c — the install point of libsvtgpu's RTCD shims (test infrastructure; never shipped).
 *
 * The encoder copies the sad / variance / highbd variance / sub-pixel variance / x4d pointers into svt_aom_mefn_ptr[]
 * once, in init_fn_ptr (av1me.c:31), called at EbEncHandle.c:1546 right after the RTCD setup (:1530-1531); ME and MD
 * then call through that table (EbProductCodingLoop.c:999, EbModeDecision.c:2185, ...).  This harness links the
 * reference's own av1me.c and aom_dsp_rtcd.c with libsvtgpu and runs include/svtgpu_rtcd.h's install both ways:
 *   documented order: svtgpu_install_me_md_rtcd() then init_fn_ptr()  -> every entry init_fn_ptr writes is a shim;
 *   late install:     init_fn_ptr() then svtgpu_install_me_md_rtcd()  -> no entry is (MD stays on the CPU).
 * Pointer comparisons only (dladdr): no device call, so it runs without a GPU.  Output: one line
 *   "documented <shims>/<entries> late <shims>/<entries>".
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
#include <string.h>

#include "EbDefinitions.h"
#include "aom_dsp_rtcd.h"
#include "common_dsp_rtcd.h"
#include "EbMcp.h"
#include "av1me.h"
#include "svtgpu_rtcd.h"

void init_fn_ptr(void);

static int in_libsvtgpu(const void *f) {
    Dl_info d;
    return f && dladdr(f, &d) && d.dli_fname && strstr(d.dli_fname, "libsvtgpu") != NULL;
}

/* entries of svt_aom_mefn_ptr[] that init_fn_ptr wrote (non-null), and how many of them are libsvtgpu shims */
static void census(int *shims, int *entries) {
    *shims = *entries = 0;
    for (int b = 0; b < BlockSizeS_ALL; b++) {
        const void *f[5] = {(const void *)svt_aom_mefn_ptr[b].sdf, (const void *)svt_aom_mefn_ptr[b].vf,
                            (const void *)svt_aom_mefn_ptr[b].vf_hbd_10, (const void *)svt_aom_mefn_ptr[b].svf,
                            (const void *)svt_aom_mefn_ptr[b].sdx4df};
        for (int k = 0; k < 5; k++)
            if (f[k]) ++*entries, *shims += in_libsvtgpu(f[k]);
    }
}

/* the C kernels the RTCD setup binds on a host without SIMD (svt_aom_setup_rtcd_internal, aom_dsp_rtcd.c) */
#define C_SIZE(w, h)                                                           \
    svt_aom_sad##w##x##h                = svt_aom_sad##w##x##h##_c;               \
    svt_aom_sad##w##x##h##x4d           = svt_aom_sad##w##x##h##x4d_c;            \
    svt_aom_variance##w##x##h           = svt_aom_variance##w##x##h##_c;          \
    svt_aom_highbd_10_variance##w##x##h = svt_aom_highbd_10_variance##w##x##h##_c; \
    svt_aom_sub_pixel_variance##w##x##h = svt_aom_sub_pixel_variance##w##x##h##_c;
static void bind_c(void) {
    C_SIZE(4, 4) C_SIZE(4, 8) C_SIZE(4, 16) C_SIZE(8, 4) C_SIZE(8, 8) C_SIZE(8, 16) C_SIZE(8, 32) C_SIZE(16, 4)
    C_SIZE(16, 8) C_SIZE(16, 16) C_SIZE(16, 32) C_SIZE(16, 64) C_SIZE(32, 8) C_SIZE(32, 16) C_SIZE(32, 32)
    C_SIZE(32, 64) C_SIZE(64, 16) C_SIZE(64, 32) C_SIZE(64, 64) C_SIZE(64, 128) C_SIZE(128, 64) C_SIZE(128, 128)
}

int main(void) {
    int s1, e1, s2, e2;
    /* the documented order: RTCD setup, install, init_fn_ptr */
    bind_c();
    svtgpu_install_me_md_rtcd();
    init_fn_ptr();
    census(&s1, &e1);
    /* a late install: init_fn_ptr has copied the setup's pointers before the shims went in */
    bind_c();
    init_fn_ptr();
    svtgpu_install_me_md_rtcd();
    census(&s2, &e2);
    printf("documented %d/%d late %d/%d\n", s1, e1, s2, e2);
    return 0;
}
