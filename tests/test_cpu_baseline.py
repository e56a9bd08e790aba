"""The reference CPU baseline (oracle/_ref/ref_bench: the reference's own C + AVX2/SSE2 kernels, built from
/root/reference by oracle/ref.mk) runs the same algorithm as the oracle: on a crop of the bench workload its DLF level
search and CDEF strength-count choice agree with oracle.dlf_pick / oracle.cdef_pick. No GPU needed; skipped where the
reference build is absent."""
import os
import re
import subprocess
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
import svtgpu  # noqa: E402
import synth  # noqa: E402

REF_BENCH = os.path.join(ROOT, "oracle", "_ref", "ref_bench")


@pytest.mark.skipif(not os.path.exists(REF_BENCH), reason="oracle/_ref/ref_bench not built (needs /root/reference)")
def test_ref_bench_agrees_with_oracle_on_a_crop():
    import bench
    W, H, bd, q, lam = 1024, 512, 10, 128, 60000
    src, rec = synth.frame_pair(W, H, bd, seed=0x5EED0003)
    mi = synth.mode_info(W, H, 3)
    ctrls = svtgpu.cdef_controls(1)
    lr_ctrls = svtgpu.lr_controls(1, 1, rdmult=7000, switchable=(300, 700, 900), wiener=(250, 800), sgrproj=(250, 900))
    refs = [synth.frame_pair(W, H, bd, seed=0x5EED0005 + 17 * (r + 1))[0][0] for r in range(2)]
    nsb = (W // 64) * (H // 64)
    mvs = np.random.default_rng(5).integers(-16, 17, size=(nsb, 2, 2))
    with tempfile.NamedTemporaryFile(suffix=".bin") as f:
        bench.write_ref_bench_input(f, src, rec, mi, ctrls, bd, q, lam, "2x1", lr_ctrls, refs, mvs, (16, 16, 8, 8))
        f.flush()
        res = subprocess.run([REF_BENCH, f.name, "2"], capture_output=True, text=True, timeout=300,
                             env=dict(os.environ, REF_BENCH_VERBOSE="1"))
    assert res.returncode == 0, res.stderr
    assert re.match(r"ref_bench px=%d seconds=[0-9.]+ threads=2" % (W * H), res.stdout)
    m = re.search(r"crop 0,0: dlf (\d+)/(\d+)/(\d+)/(\d+) cdef sb (\d+) nbits (\d+)", res.stderr)
    assert m, res.stderr
    ref_lv, ref_sb, ref_bits = [int(m.group(k)) for k in range(1, 5)], int(m.group(5)), int(m.group(6))
    # the oracle on the same crop (512 x 512 at the origin)
    cw, ch = 512, 512
    mi_c = np.ascontiguousarray(mi[:ch // 4, :cw // 4])
    crop = [np.ascontiguousarray(rec[0][:ch, :cw])] + [np.ascontiguousarray(p[:ch // 2, :cw // 2]) for p in rec[1:]]
    cs = [np.ascontiguousarray(src[0][:ch, :cw])] + [np.ascontiguousarray(p[:ch // 2, :cw // 2]) for p in src[1:]]
    lfp = oracle.dlf_pick(crop, cs, bd, mi_c, svtgpu.LfParams.make(16, 16, 8, 8), 0, 0, 0, 0, 0)
    assert ref_lv == [lfp.filter_level[0], lfp.filter_level[1], lfp.filter_level_u, lfp.filter_level_v]
    crop = oracle.dlf_frame(crop, bd, mi_c, lfp)
    oc = oracle.controls(1)
    mse, skip, _, _ = oracle.cdef_search_frame(crop, cs, bd, oc, q)
    prm, _ = oracle.cdef_pick(cw, ch, mse, skip, oc, q, lam)
    assert ref_sb == int((np.asarray(skip) == 0).sum())
    assert ref_bits == prm.cdef_bits
