"""How many self-guided eps could an exact bound-ordered search skip?  (The verdict's round-4 item 1: measure the
prunable fraction with the oracle first.)

For the luma restoration units of a pipeline case (default c3_4k10: the bench frame), the oracle's CDEF output
(oracle/ pipeline up to the CDEF apply) is searched by oracle_lr_sgr_probe: per unit and ep the exact error of
search_sgr (EbRestorationPick.c:550-652) and the lower bound err >= (sqrt(Qmin) - sqrt(N)/2)^2 valid for any xq.
Reported: (a) the ideal fraction -- eps whose bound is above the unit's best error (no order can evaluate fewer);
(b) a bound-ordered search -- eps evaluated in ascending bound until the next bound exceeds the best error so far.
usage: sgr_prune_probe.py [case] [--cache file.npz]"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "svt-av1_pro-anchor-v2.1.0-_amd")]


def oracle_to_cdef(case):
    """tests/pipeline_run.run_oracle up to the CDEF apply (the LR search's input)."""
    import oracle
    import pipeline_cases as pc
    import pipeline_run as pr
    c, g = pc.CASES[case], pc.load(case)
    src, rec, mi = pc.inputs(case)
    bd, w, h = c["bd"], c["w"], c["h"]
    dc = pr.dlf_ctrls(c["dlf_level"])
    if dc["sb_based"]:
        lfp = pr.sb_dlf_params(c, [int(x) for x in g["lf_levels"]])
    else:
        lfp = oracle.dlf_pick(rec, src, bd, mi, pc.lf_params(c), dc["avg"], dc["avg_uv"], c["tl"], dc["early_exit"],
                              c["only4x4"])
    dlf = oracle.dlf_frame(rec, bd, mi, lfp)
    print("dlf done", flush=True)
    mask = pc.cdef_mask(mi)
    ctrls = oracle.controls(c["cdef_level"])
    ctrls.pred_y_f, ctrls.pred_uv_f = c["pred"]
    nvfb, nhfb = (((h + 7) & ~7) // 4 + 15) // 16, (((w + 7) & ~7) // 4 + 15) // 16
    fbb = np.ascontiguousarray(mi)["bsize"][::16, ::16].reshape(-1) if c["sb"] == 128 else None
    mse, skip, d, v = oracle.cdef_search_frame(dlf, src, bd, ctrls, c["q"], mask, fbb)
    print("cdef search done", flush=True)
    kinds = oracle.cdef_fb_kinds(fbb, nvfb, nhfb) if fbb is not None else None
    prm, fbs = oracle.cdef_pick(w, h, mse, skip, ctrls, c["q"], int(g["cdef_lambda"][0]))
    if kinds is not None:
        fbs = oracle.cdef_dup_sb128(fbs, kinds, nvfb, nhfb)
    nb = 1 << prm.cdef_bits
    applied = int(prm.cdef_y_strength[0] != 0 or prm.cdef_uv_strength[0] != 0 or nb != 1)
    cdef = oracle.cdef_apply_frame(dlf, bd, mask, d, v, prm, fbs) if applied else [p.copy() for p in dlf]
    return src, cdef


def main():
    case = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "c3_4k10"
    cache = sys.argv[sys.argv.index("--cache") + 1] if "--cache" in sys.argv else "/tmp/sgr_probe_%s.npz" % case
    import oracle
    import pipeline_cases as pc
    c = pc.CASES[case]
    t0 = time.time()
    if os.path.exists(cache):
        z = np.load(cache)
        cdef0, src0 = z["cdef0"], z["src0"]
    else:
        src, cdef = oracle_to_cdef(case)
        cdef0, src0 = np.ascontiguousarray(cdef[0], np.uint16), np.ascontiguousarray(src[0], np.uint16)
        np.savez(cache, cdef0=cdef0, src0=src0)
    print("inputs %.1f s" % (time.time() - t0), flush=True)
    lrc = oracle.lr_controls(c["wn_level"], c["sg_level"], c["rdmult"], c["sw"], c["wc"], c["sc"])
    start, end, inc, refine = lrc.sg_start_ep[0], lrc.sg_end_ep[0], lrc.sg_ep_inc[0], lrc.sg_refine[0]
    neps = len(range(start, end, inc))
    h, w = cdef0.shape
    usz = c["us"][0]
    nmax = ((w + usz - 1) // usz + 1) * ((h + usz - 1) // usz + 1)
    err = np.zeros((nmax, neps), np.int64)
    bnd = np.zeros((nmax, neps), np.float64)
    f = oracle.lib().oracle_lr_sgr_probe
    f.restype = ctypes.c_int
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    t0 = time.time()
    n = f(P(cdef0), ctypes.c_int(w), P(src0), ctypes.c_int(w), w, h, c["bd"], usz, start, end, inc, refine, P(err), P(bnd))
    err, bnd = err[:n], bnd[:n]
    print("probe: %d units x %d eps (eps %d..%d step %d, refine %d), %.1f s" % (n, neps, start, end, inc, refine,
                                                                           time.time() - t0))
    best = err.min(axis=1)
    assert (bnd <= err + 1e-6).all(), "bound above an exact error"
    ideal = (bnd > best[:, None]).sum()
    evals = 0
    for u in range(n):
        order = np.argsort(bnd[u], kind="stable")
        cur = None
        for k in order:
            if cur is not None and bnd[u, k] > cur:
                break
            evals += 1
            cur = err[u, k] if cur is None else min(cur, err[u, k])
    slack = np.sqrt(err) - np.sqrt(bnd)
    print("ideal prunable: %d of %d (%.1f %%); bound-ordered search evaluates %d (%.1f %%)" %
          (ideal, err.size, 100.0 * ideal / err.size, evals, 100.0 * evals / err.size))
    print("best err per unit: median %.0f (sqrt %.0f); sqrt(err) - sqrt(bound): median %.1f" %
          (np.median(best), np.sqrt(np.median(best)), np.median(slack)))
    print("err / best per ep (median over units):", np.round(np.median(err / best[:, None], axis=0), 3).tolist())


if __name__ == "__main__":
    main()
