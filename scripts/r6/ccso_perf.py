"""CCSO on the MI355X: one frame's ccso_search (the three planes' derive_ccso_filter) and ccso_frame
(the three planes' apply), device-resident inputs, timed with HIP events on the library stream; the bins pass's
roofline; the reference's own CPU search beside it (oracle/_ref/gen_golden_ccso bench, AVX2 kernels, one thread) when
that binary is present.  One JSON line per size.

    python3 scripts/r6/ccso_perf.py [--sizes 1920x1080x8,3840x2160x10] [--reps 10] [--cpu]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import svtgpu  # noqa: E402

HBM_PEAK = 8000.0  # GB/s, MI355X_MICROARCH.md


def content(w, h, bd, seed):
    """the parity tests' content model (tests/ccso_cases.py:content): smooth org, band / edge biased coding error"""
    import ccso_cases
    return ccso_cases.content(w, h, bd, seed)


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).cuda()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1920x1080x8,3840x2160x10")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu", action="store_true", help="also time the reference's CPU search (AVX2, one thread)")
    args = ap.parse_args()
    ctx = svtgpu.Context(0)
    stream = torch.cuda.ExternalStream(ctx.stream)
    for spec in args.sizes.split(","):
        w, h, bd = (int(v) for v in spec.split("x"))
        org, rec, pre = content(w, h, bd, seed=w + h)
        st = svtgpu.CcsoState(ctx, w, h)
        d_org, d_rec, d_pre = [dev(a) for a in org], [dev(a) for a in rec], dev(pre)
        ext = torch.zeros(((h + 10) * (w + 10),), dtype=torch.int16, device="cuda")
        planes = [dev(rec[p][: (h >> 1 if p else h), : (w >> 1 if p else w)].copy()) for p in range(3)]
        torch.cuda.synchronize()
        rdmult, q = 1500, 100

        def search():  # ccso_search: the padded luma, then the three planes' searches in one launch per pass
            st.extend(d_pre.data_ptr(), 16, w, ext.data_ptr())
            st.search_frame(ext.data_ptr(), [t.data_ptr() for t in d_org], [t.data_ptr() for t in d_rec], bd, rdmult,
                            q, read=False)

        def apply():
            for p in range(3):
                st.apply(ext.data_ptr(), p, bd, planes[p].data_ptr(), 16, planes[p].shape[1])

        for _ in range(3):
            search(), apply()
        ctx.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        with torch.cuda.stream(stream):
            ev[0].record()
            for _ in range(args.reps):
                search()
            ev[1].record()
            for _ in range(args.reps):
                apply()
            ev[2].record()
        ev[2].synchronize()
        ms_search, ms_apply = ev[0].elapsed_time(ev[1]) / args.reps, ev[1].elapsed_time(ev[2]) / args.reps
        prm = [p.fields() for p in st.search_frame(ext.data_ptr(), [t.data_ptr() for t in d_org],
                                                   [t.data_ptr() for t in d_rec], bd, rdmult, q)[1]]
        px = w * h * 3 // 2
        # compulsory bytes of the search: org + rec of every plane sample (2 + 2 B) + the padded luma (2 B per luma
        # sample, read by the luma and both chroma passes); the apply: each plane sample read and written + the luma
        search_bytes = 4 * px + 2 * (w + 10) * (h + 10)
        apply_bytes = 2 * 2 * px + 2 * w * h
        line = {"metric": "ccso_search_frames_per_s", "w": w, "h": h, "bd": bd, "reps": args.reps,
                "search_ms": round(ms_search, 3), "apply_ms": round(ms_apply, 4),
                "search_mpx_s": round(px / ms_search / 1e3, 1), "apply_gb_s": round(apply_bytes / ms_apply / 1e6, 1),
                "search_compulsory_gb_s": round(search_bytes / ms_search / 1e6, 1), "hbm_peak_gb_s": HBM_PEAK,
                "params": prm, "data": "synthetic (tests/ccso_cases.py content model)"}
        if args.cpu:
            exe = os.path.join(ROOT, "oracle", "_ref", "gen_golden_ccso")
            if os.path.exists(exe):
                t0 = time.time()
                out = subprocess.run([exe, "bench", str(w), str(h), str(bd), "1", "avx2"], capture_output=True,
                                     text=True, timeout=600).stdout
                ref = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
                line["cpu_baseline"] = {"search_ms": ref["search_ms"], "apply_ms": ref["apply_ms"], "cores": 1,
                                        "kind": "reference", "kernels": "avx2",
                                        "sample": "one frame, ccso_search + ccso_frame (8-bit only)",
                                        "wall_s": round(time.time() - t0, 1)}
                line["speedup_search"] = round(ref["search_ms"] / ms_search, 1)
        print(json.dumps(line), flush=True)
        st.close()


if __name__ == "__main__":
    main()
