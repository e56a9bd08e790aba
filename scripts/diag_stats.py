"""Diagnostic: run the compute_stats shim on every lr_stats.bin case several times and report mismatches."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd"), os.path.join(ROOT, "tests")]
import svtgpu, cdef_cases as cc
ctx = svtgpu.Context(0)
L, g = svtgpu.lib(), cc.load("lr_stats.bin")
addr = lambda a, o=0: ctypes.c_void_p(a.ctypes.data + o * a.itemsize)
byteptr = lambda a, o=0: ctypes.c_void_p((a.ctypes.data + o * a.itemsize) >> 1)
for rep in range(3):
    for n in range(len(g["meta"])):
        bd, win, w, h, st, _ = (int(x) for x in g["meta"][n])
        d, s = np.ascontiguousarray(g["dgd%d" % n]), np.ascontiguousarray(g["src%d" % n])
        M, H = np.zeros(win * win, np.int64), np.zeros(win ** 4, np.int64)
        o = 4 * st + 4
        if bd == 8:
            d8, s8 = d.astype(np.uint8), s.astype(np.uint8)
            L.svtgpu_av1_compute_stats(win, addr(d8, o), addr(s8, o), 0, w, 0, h, st, st, addr(M), addr(H))
        else:
            L.svtgpu_av1_compute_stats_highbd(win, byteptr(d, o), byteptr(s, o), 0, w, 0, h, st, st, addr(M), addr(H), bd)
        okm, okh = np.array_equal(M, g["M%d" % n]), np.array_equal(H, g["H%d" % n])
        print(rep, n, (bd, win, w, h, st), "M ok" if okm else "M BAD %s vs %s" % (M[:3], g["M%d" % n][:3]),
              "H ok" if okh else "H BAD", d.dtype, flush=True)
