"""rest_finish_search (EbRestorationPick.c:1555-1634) on the host side of the C ABI, against the reference's own
outputs (tests/golden/lr_search.bin, gen_golden_lr.c): the per-unit search records the reference's
restoration_seg_search left in rusi_picture go through svtgpu_lr_finish_frame, whose frame types and unit
parameters must equal what the reference's rest_finish_search chose.  Cases 10-13 search one filter type for luma
only (Wiener level 5 beside self-guided level 3 / 1, self-guided level 4 beside Wiener level 1): the reference's
RestUnitSearchInfo array is shared by the planes, so a chroma plane's switchable pass reads luma's entries for the
type chroma does not search (c13: a chroma unit takes the Wiener filter from luma's entry).  No device is touched.
The device form of the same finish (lr_fin_*_kernel) is compared with these fixtures in tests/test_lr_gpu.py."""
import numpy as np
import pytest

import lr_cases as lc
import svtgpu

CASES = list(lc.search_cases())


def _records(c):
    """The reference's per-unit search records of case c as SvtGpuLrUnitSearch arrays."""
    out = []
    for p in range(3):
        sse, rp = c["sse"][p], c["rec_params"][p]
        r = np.zeros(len(sse), svtgpu.LR_UNIT_SEARCH_DTYPE)
        s = sse.copy()
        s[s == -1] = np.iinfo(np.int64).max
        r["sse"] = s
        r["wiener"]["type"] = 1
        r["wiener"]["vfilter"] = rp[:, 0:8]
        r["wiener"]["hfilter"] = rp[:, 8:16]
        r["sgrproj"]["type"] = 2
        r["sgrproj"]["ep"] = rp[:, 16]
        r["sgrproj"]["xqd"] = rp[:, 17:19]
        out.append(r)
    return out


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_finish_frame_vs_reference(ci):
    c = CASES[ci]
    ctrls = c["ctrls"]
    recs = _records(c)
    ft, units = svtgpu.lr_finish_frame(ctrls, recs)
    lc.compare_search(ft, units, None, c)


def test_leftover_case_needs_the_shared_array():
    """c13 (328x184, Wiener level 5 + self-guided level 3): finishing the chroma planes one by one (no luma entries)
    gives another answer than the reference, the shared-array finish gives the reference's."""
    c = next(x for x in CASES if x["name"].startswith("c13_"))
    recs = _records(c)
    ft, units = svtgpu.lr_finish_frame(c["ctrls"], recs)
    lc.compare_search(ft, units, None, c)
    alone = [svtgpu.lr_finish_plane(c["ctrls"], p, recs[p]) for p in range(3)]
    assert any(not np.array_equal(alone[p][1]["type"], c["units"][p]["type"]) for p in (1, 2))
