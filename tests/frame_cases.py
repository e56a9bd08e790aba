"""Frame-buffer test helpers: the reference goldens (tests/golden/frame_ops.bin, oracle/ref_harness/gen_golden_frame.c)."""
import cdef_cases as cc


def golden():
    return cc.load("frame_ops.bin")


def conv_cases(g):
    """(src, dst_before, dst_after, w, h, src_stride, dst_stride)"""
    return [(g["conv_src%d" % n], g["conv_dst0_%d" % n], g["conv_dst%d" % n], *[int(v) for v in m[:4]])
            for n, m in enumerate(g["meta"][0])]


def pad_cases(g):
    """(before, after, w, h, stride, pw, ph)"""
    return [(g["pad_in%d" % n], g["pad_out%d" % n], *[int(v) for v in m[:5]]) for n, m in enumerate(g["meta"][1])]


def ext_cases(g):
    """(before, after, w, h, stride, bh, bv, offset of the first visible sample)"""
    return [(g["ext_in%d" % n], g["ext_out%d" % n], int(m[0]), int(m[1]), int(m[2]), int(m[3]), int(m[4]), int(m[6]))
            for n, m in enumerate(g["meta"][2])]
