"""Build-time edit of a /tmp copy of the reference's EbCdefProcess.c for the drop-in encoder (test infrastructure;
oracle/enc.mk target libsvtenc_nss.so, tests/test_encoder_drop_in.py): the CDEF process body's per-segment CPU strength
search -- the one call of the static cdef_seg_search in svt_aom_cdef_kernel (EbCdefProcess.c:400-404) -- is removed, so
an encoder whose finish_cdef_search is served by the device (enc_frame_hooks.c: svtgpu_cdef_search_frame over the
whole frame + svtgpu_cdef_pick) no longer runs the CPU search beside it.  That is INTEGRATION.md §2's integration
applied to the process body.  The copy is written outside the repository and only its object file is kept
(oracle/_ref/enc); no reference text is stored in the repository.

usage: no_seg_search.py <EbCdefProcess.c> <out.c>
"""
import re
import sys

src, out = sys.argv[1], sys.argv[2]
text = open(src).read()
call = re.compile(r"^([ \t]*)cdef_seg_search\(\s*pcs\s*,\s*scs\s*,\s*dlf_results->segment_index\s*\)\s*;", re.M)
hits = call.findall(text)
if len(hits) != 1:
    sys.exit("no_seg_search: expected exactly one call of cdef_seg_search in %s, found %d" % (src, len(hits)))
text = call.sub(r"\1/* per-segment CPU search removed: the device searches the whole frame in finish_cdef_search */ "
                r"(void)scs;", text)
# the function itself is left in place (static, now unreferenced: the compiler drops it)
with open(out, "w") as f:
    f.write('#line 1 "%s"\n' % src)
    f.write(text)
