"""Summarise the per-workgroup clocks that SVTGPU_WGCLK=<file> records (svtgpu_internal.h wgclk_mark).
usage: wgclk.py <file> [kernel]   -- per launch: span, WG duration percentiles, start ramp, per-XCC counts"""
import sys

import numpy as np


def launches(path):
    raw = open(path, "rb").read()
    o = 0
    while o < len(raw):
        name = raw[o:o + 64].split(b"\0")[0].decode()
        n = int(np.frombuffer(raw, np.int64, 1, o + 64)[0])
        a = np.frombuffer(raw, np.uint64, 4 * n, o + 72).reshape(n, 4).astype(np.int64)
        o += 72 + 32 * n
        yield name, a


def main(path, only=None):
    per = {}
    for name, a in launches(path):
        if only and name != only:
            continue
        ok = a[:, 1] > 0
        t0 = a[:, 0].min()
        span = (a[ok, 1].max() - t0) * 10.0  # 100 MHz ticks -> ns
        dur = (a[ok, 1] - a[ok, 0]) * 10.0
        start = (a[:, 0] - t0) * 10.0
        xcc = a[:, 3] & 0xF
        per.setdefault(name, []).append((span, np.percentile(dur, [10, 50, 90, 100]), np.percentile(start, [50, 90, 100]),
                                         np.bincount(xcc, minlength=8)[:8], len(a)))
    for name, rows in per.items():
        print("%s: %d launches" % (name, len(rows)))
        for span, d, s, x, n in rows[:6] + ([] if len(rows) <= 6 else rows[-2:]):
            print("  n=%5d span %7.1f us | WG dur p10/50/90/max %6.1f %6.1f %6.1f %6.1f us | start p50/90/max %6.1f %6.1f "
                  "%6.1f us | per XCC %s" % (n, span / 1e3, *(d / 1e3), *(s / 1e3), x.tolist()))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
