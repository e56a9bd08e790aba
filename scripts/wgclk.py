"""Summarise the per-workgroup clocks that SVTGPU_WGCLK=<file> records (svtgpu_internal.h wgclk_mark: 8 words per
workgroup -- time marks 0..5 on the 100 MHz clock, 0 where unused; HW_ID; XCC_ID).
usage: wgclk.py <file> [kernel]   -- per launch: span, start ramp, workgroup duration and per-phase percentiles"""
import sys

import numpy as np


def launches(path):
    raw = open(path, "rb").read()
    o = 0
    while o < len(raw):
        name = raw[o:o + 64].split(b"\0")[0].decode()
        n = int(np.frombuffer(raw, np.int64, 1, o + 64)[0])
        a = np.frombuffer(raw, np.uint64, 8 * n, o + 72).reshape(n, 8).astype(np.int64)
        o += 72 + 64 * n
        yield name, a


def pct(x):
    return "%6.1f/%6.1f/%6.1f" % tuple(np.percentile(x, [10, 50, 90])) if len(x) else "     -"


def main(path, only=None, show=6):
    per = {}
    for name, a in launches(path):
        if not only or name == only:
            per.setdefault(name, []).append(a)
    for name, rows in per.items():
        print("%s: %d launches (us; p10/p50/p90)" % (name, len(rows)))
        for a in rows[:show] + (rows[-2:] if len(rows) > show else []):
            a = a[a[:, 0] > 0]  # workgroups that recorded a start
            t0 = a[:, 0].min()
            last = np.where(a[:, 1:6] > 0, a[:, 1:6], 0).max(axis=1)  # the workgroup's last mark
            done = last > 0
            span = (last.max() - t0) / 100.0
            out = ["n=%5d span %7.1f start %s dur %s" % (len(a), span, pct((a[:, 0] - t0) / 100.0),
                                                         pct((last[done] - a[done, 0]) / 100.0))]
            prev = a[:, 0]
            for k in range(1, 6):
                m = a[:, k] > 0
                if m.any():
                    out.append("ph%d %s" % (k, pct((a[m, k] - prev[m]) / 100.0)))
                    prev = np.where(m, a[:, k], prev)
            print("  " + " | ".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
