"""Build-time edit of a /tmp copy of the reference's EbCdefProcess.c for the drop-in encoder (test infrastructure;
oracle/enc.mk target oracle/_ref/enc/ccso/, tests/test_encoder_drop_in.py): the fork's CCSO search and apply, which
its CDEF process body carries commented out after finish_cdef_search / svt_av1_cdef_frame (EbCdefProcess.c:621-623;
the buffers they read are still built around them, :414-503 and :524-661), are switched back on -- the two comment
markers removed, nothing else changed.  That encoder is the reference CPU path of SURVEY §8(f)4; with the CCSO hooks
(enc_frame_hooks.c) its ccso_search / ccso_frame calls land on the device.  The copy is written outside the repository
and only its object file is kept (oracle/_ref/enc/ccso); no reference text is stored in the repository.

usage: with_ccso.py <EbCdefProcess.c> <out.c>
"""
import re
import sys

src, out = sys.argv[1], sys.argv[2]
text = open(src).read()
calls = [r"ccso_search\(\s*pcs\s*,\s*pd\s*,\s*\(int\)\s*lambda\s*,\s*ext_rec_y\s*,\s*rec_uv\s*,\s*org_uv\s*\)\s*;",
         r"ccso_frame\(\s*recon_pic\s*,\s*pcs\s*,\s*pd\s*,\s*ext_rec_y\s*\)\s*;"]
for c in calls:
    pat = re.compile(r"^([ \t]*)//[ \t]*(" + c + r")", re.M)
    hits = pat.findall(text)
    if len(hits) != 1:
        sys.exit("with_ccso: expected exactly one commented call matching %s in %s, found %d" % (c, src, len(hits)))
    text = pat.sub(r"\1\2", text)
with open(out, "w") as f:
    f.write('#line 1 "%s"\n' % src)
    f.write(text)
