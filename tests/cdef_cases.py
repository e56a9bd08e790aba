"""Helpers that turn golden CDEF fixtures into call arguments (shared by CPU and GPU tests)."""
import ctypes
import os

import numpy as np

import golden_io

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BSTRIDE = 144


def load(name):
    return golden_io.load(os.path.join(GOLDEN, name))


def filter_block_case(g, n):
    """Expand the 12x12 window of case n into a 144-stride CDEF input buffer; returns (buf, in_offset, params)."""
    win = g["win"][n].reshape(12, 12)
    buf = np.full(BSTRIDE * 20, 0x7F7F, np.uint16)
    off = 4 * BSTRIDE + 8  # block origin: row 4, col 8 of the buffer
    for i in range(12):
        buf[off + (i - 2) * BSTRIDE - 2: off + (i - 2) * BSTRIDE + 10] = win[i]
    return buf, off, [int(x) for x in g["params"][n]]


def run_filter_block(fn, g, n):
    buf, off, (bd, bsize, pri, sec, d, pdamp, sdamp, ss, use8, _b) = filter_block_case(g, n)
    bw = 8 if bsize in (2, 3) else 4
    inp = ctypes.c_void_p(buf.ctypes.data + 2 * off)
    if use8:
        dst = np.full(64, 0xA5, np.uint8)
        fn(ctypes.c_void_p(dst.ctypes.data), None, bw, inp, pri, sec, d, pdamp, sdamp, bsize, bd - 8, ss)
        return dst.astype(np.uint16)
    dst = np.full(64, 0xA5A5, np.uint16)
    fn(None, ctypes.c_void_p(dst.ctypes.data), bw, inp, pri, sec, d, pdamp, sdamp, bsize, bd - 8, ss)
    return dst


def run_cdef_dist(fn16, fn8, g, n):
    bd, bsize, count, pli, ss, is8 = [int(x) for x in g["params"][n]]
    src = g["src"][n]
    flt = g["flt"][n]
    dl = np.ascontiguousarray(g["dlist"][n][:2 * count])
    st = 68
    if is8:
        s8 = np.ascontiguousarray(src.astype(np.uint8))
        f8 = np.ascontiguousarray(flt.astype(np.uint8))
        return fn8(ctypes.c_void_p(s8.ctypes.data), st, ctypes.c_void_p(f8.ctypes.data),
                   ctypes.c_void_p(dl.ctypes.data), count, bsize, bd - 8, pli, ss)
    s16 = np.ascontiguousarray(src)
    f16 = np.ascontiguousarray(flt)
    return fn16(ctypes.c_void_p(s16.ctypes.data), st, ctypes.c_void_p(f16.ctypes.data),
                ctypes.c_void_p(dl.ctypes.data), count, bsize, bd - 8, pli, ss)


def run_search_one_dual(fn, g, n):
    mse = np.ascontiguousarray(g["mse"][n])  # [2][SB][64]
    nb, start, end = [int(x) for x in g["params"][n]]
    sb = mse.shape[1]
    U64P = ctypes.POINTER(ctypes.c_uint64)
    rows = [(U64P * sb)(*[ctypes.cast(mse[p, i].ctypes.data, U64P) for i in range(sb)]) for p in range(2)]
    arr = (ctypes.POINTER(U64P) * 2)(*[ctypes.cast(r, ctypes.POINTER(U64P)) for r in rows])
    l0 = (ctypes.c_int * 16)(*[int(x) for x in g["lev_in"][n][0]])
    l1 = (ctypes.c_int * 16)(*[int(x) for x in g["lev_in"][n][1]])
    best = fn(l0, l1, nb, arr, sb, start, end)
    return best, list(l0), list(l1), mse
