/*
 * ref_cdef_process.c — test infrastructure (golden generation only; never shipped, never on the product path).
 *
 * cdef_seg_search (Source/Lib/Encoder/Codec/EbCdefProcess.c:114) has internal linkage, so this harness unit is
 * compiled together with the reference's own EbCdefProcess.c, as it lies under /root/reference (the include
 * resolves through ref.mk's -I paths), and forwards to it under a harness name.  --gc-sections drops the parts
 * of that unit the generator never reaches.
 */
#include "EbCdefProcess.c"

void ref_cdef_seg_search(PictureControlSet *pcs, SequenceControlSet *scs, uint32_t segment_index) {
    cdef_seg_search(pcs, scs, segment_index);
}
