/*
 * ref_mode_config.c — test infrastructure (golden generation only; never shipped, never on the product path).
 *
 * The encoder's per-level control tables for the hot path live in static functions of the reference's
 * EncModeConfig.c: set_cdef_controls (:860), svt_aom_set_wn_filter_ctrls (:1329), svt_aom_set_sg_filter_ctrls
 * (:1386) and svt_aom_set_dlf_controls (:1557).  This unit is compiled together with that file, as it lies under
 * /root/reference, so the pipeline generator reads the controls from the reference itself rather than from a
 * restatement; --gc-sections drops everything else in it.
 */
#include "EncModeConfig.c"

void ref_set_cdef_controls(PictureParentControlSet *pcs, uint8_t cdef_level, int fast_decode) {
    set_cdef_controls(pcs, cdef_level, fast_decode);
}
void ref_set_wn_filter_ctrls(Av1Common *cm, uint8_t lvl) { svt_aom_set_wn_filter_ctrls(cm, lvl); }
void ref_set_sg_filter_ctrls(Av1Common *cm, uint8_t lvl) { svt_aom_set_sg_filter_ctrls(cm, lvl); }
void ref_set_dlf_controls(PictureParentControlSet *pcs, uint8_t lvl) { svt_aom_set_dlf_controls(pcs, lvl); }
