"""bench.py times the reference-pinned frames: its PINNED inputs and frame-level controls are those of the pipeline
cases whose reference outputs tests/test_pipeline_golden.py checks the GPU against (the benched frames
must be the pinned frames)."""
import numpy as np
import pytest

import bench
import pipeline_cases as pc
import synth


@pytest.mark.parametrize("key", sorted(bench.PINNED))
def test_pinned_bench_config_is_the_golden_case(key):
    w, h, bd = key
    b = bench.PINNED[key]
    c = pc.CASES[b["case"]]
    g = pc.load(b["case"])
    assert (c["w"], c["h"], c["bd"]) == (w, h, bd)
    assert b["seed"] == c["seed"] and b["q"] == c["q"] and tuple(b["lf"]) == tuple(c["lf"])
    assert b["lam"] == int(g["cdef_lambda"][0])
    assert b["rdmult"] == c["rdmult"] and tuple(b["sw"]) == tuple(c["sw"]) and tuple(b["wc"]) == tuple(c["wc"])
    assert tuple(b["sc"]) == tuple(c["sc"]) and tuple(b["us"]) == tuple(c["us"])
    assert c["mi"][0] == "bench" and c["cdef_level"] == 1 and c["dlf_level"] == 1
    assert (c["wn_level"], c["sg_level"], c["mrd"], c["sharp"], c["sb"]) == (1, 1, 0, 0, 64)
    import pipeline_run
    d = pipeline_run.dlf_ctrls(c["dlf_level"])  # bench.py's pick: dlf_avg = dlf_avg_uv = early_exit = 0, layer 0
    assert (d["avg"], d["avg_uv"], d["early_exit"], c["tl"], c["only4x4"]) == (0, 0, 0, 0, 0)


def test_pinned_inputs_digest():
    """The frames bench.py generates for the 4K 10-bit line hash to the fixture's input digest."""
    b = bench.PINNED[(3840, 2160, 10)]
    src, rec = synth.frame_pair_int(3840, 2160, 10, b["seed"])
    mi = synth.mode_info(3840, 2160, 3)
    assert pc.input_digest(src, rec, mi) == str(pc.load(b["case"])["input_sha"])
