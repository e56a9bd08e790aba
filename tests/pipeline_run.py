"""Run a pipeline case (tests/pipeline_cases.py) through the GPU library or the CPU oracle and compare the result
with the reference's stored outputs (tests/golden/pipe_<case>.npz).

Both runners follow the encoder's order (EbDlfProcess.c:96-136 -> EbCdefProcess.c:398-520 ->
EbRestProcess.c:552-630): DLF level pick on the EncDec recon, filter; CDEF search on the deblocked frame, strength
pick with the reference's lambda, apply when a strength is non-zero; LR search on the CDEF output, apply with
stripe boundaries from the deblocked and CDEF frames.  The comparison is bit-exact; entries the reference never
writes (filter blocks it skips, strengths beyond the level's count, 8x8 blocks off the CDEF list) are zeroed
on both sides, and the zero-strength cost bias finish_cdef_search applies in place (EbEncCdef.c:830-836) is
applied to ours before comparing the tables.
"""
import numpy as np

import golden_io
import pipeline_cases as pc

_CTRLS = None


def ctrl_tables():
    global _CTRLS
    if _CTRLS is None:
        _CTRLS = golden_io.load(pc.os.path.join(pc.GOLDEN, "ctrls.bin"))
    return _CTRLS


def dlf_ctrls(level):
    e = ctrl_tables()["dlf"][level]
    return dict(enabled=int(e[0]), sb_based=int(e[1]), avg=int(e[2]), avg_uv=int(e[3]), early_exit=int(e[4]),
                zero_lvl=int(e[5]))


def nsb64(c):
    return ((c["w"] + 63) // 64) * ((c["h"] + 63) // 64)


def sb_dlf_params(c, levels):
    """The loop-filter parameters of the SB-based DLF levels (3-5): svt_av1_pick_filter_level(LPF_PICK_FROM_Q) sets the
    four levels and zeroes the sharpness (EbDeblockingFilter.c:1147-1150); the per-SB filter of the encode loop
    (svt_aom_loop_filter_sb in raster order, EbCodingLoop.c:2260-2281) equals the frame filter with those levels:
    an edge's filter never reads or writes samples past its neighbouring blocks, so no edge sees another's output
    within a direction whatever the SB order, and every vertical edge of an SB is filtered before the horizontal
    edges that read its samples in both orders."""
    from svtgpu import LfParams
    if c["mrd"]:
        return LfParams.make(*levels, 0, ref_deltas=c["ref_deltas"], mode_deltas=c["mode_deltas"])
    return LfParams.make(*levels, 0)


def gpu_dlf_pick(dl, R, S, c):
    """The frame's loop-filter levels on libsvtgpu: the device level search (DLF levels 1, 2) or LPF_PICK_FROM_Q (the
    SB-based levels 3-5: every SB's ME distortion the case's `mesad`, no listed references)."""
    import svtgpu
    dc = dlf_ctrls(c["dlf_level"])
    if dc["sb_based"]:
        return sb_dlf_params(c, svtgpu.dlf_pick_by_q(c["bd"], c["q"], c["frame_type"], c["slice"], c["tl"], c["tl"],
                                                     c["in_res"], dc["zero_lvl"], [c["mesad"]] * nsb64(c), []))
    return dl.pick(R, S, pc.lf_params(c), dc["avg"], dc["avg_uv"], c["tl"], dc["early_exit"], c["only4x4"])


def cdef_ctrl_row(level):
    e = ctrl_tables()["cdef"][level]
    return dict(enabled=int(e[0]), n1=int(e[1]), n2=int(e[2]), ref_fs=int(e[3]), bias=int(e[6]))


# --------------------------------------------------------------------------- reference layout of the CDEF tables
def fb_kinds(mi, nvfb, nhfb):
    """Per 64x64 filter block: 0 plain, 1 top-left of a 128x128, 2 left of a 128x64, 3 top of a 64x128, and -1 for
    the halves the reference's search skips (EbCdefProcess.c:193-196)."""
    bs = np.ascontiguousarray(mi)["bsize"]
    k = np.zeros((nvfb, nhfb), np.int8)
    for r in range(nvfb):
        for c in range(nhfb):
            b = int(bs[16 * r, 16 * c])
            if ((c & 1) and b in (15, 14)) or ((r & 1) and b in (15, 13)):
                k[r, c] = -1
            elif b in (13, 14, 15):
                k[r, c] = {15: 1, 14: 2, 13: 3}[b]
    return k.reshape(-1)


def reference_layout(case, mi, mse, skip, d, v, fbs, prm, applied):
    """Map a search result in our layout (mse [2][nfb][64], skip [nfb], dir/var [nfb][64] per 64x64 filter block) to
    the reference's tables as they stand after svt_av1_cdef_frame: mse/skip with the entries the reference never
    writes zeroed (use_reference_cdef_fs: no search at all) and the zero-strength bias applied; dir/var as
    CDEF_NBLOCKS x CDEF_NBLOCKS (16 x 16) per filter block holding every listed 8x8 block of the block's search area
    (128-wide areas for SB128 blocks), plus the directions the apply finds itself where the search left none
    (the skipped halves of SB128 areas, every block with use_reference_cdef_fs; dirinit = 0, EbEncCdef.c:403-414)."""
    c = pc.CASES[case]
    w, h = c["w"], c["h"]
    mr, mcol = ((h + 7) & ~7) >> 2, ((w + 7) & ~7) >> 2
    nvfb, nhfb = (mr + 15) // 16, (mcol + 15) // 16
    nfb = nvfb * nhfb
    ctl = cdef_ctrl_row(c["cdef_level"])
    kinds = fb_kinds(mi, nvfb, nhfb) if c["sb"] == 128 else np.zeros(nfb, np.int8)
    mse = np.array(mse, np.uint64, copy=True)
    skip = np.array(skip, np.uint8, copy=True)
    if ctl["ref_fs"]:
        mse[:] = 0
        skip[:] = 0
        searched = np.zeros(nfb, bool)
    else:
        mse[:, :, ctl["n1"] + ctl["n2"]:] = 0
        skip[kinds < 0] = 0
        searched = (kinds >= 0) & (skip == 0)
        mse[:, ~searched, :] = 0
        if ctl["bias"]:
            mse[:, searched, 0] = (np.uint64(ctl["bias"]) * mse[:, searched, 0]) >> np.uint64(6)
    mask = pc.cdef_mask(mi)
    nby, nbx = mask.shape
    D = np.zeros((nvfb * 8, nhfb * 8), np.uint8)  # frame grid of our per-filter-block tables
    V = np.zeros((nvfb * 8, nhfb * 8), np.int32)
    for f in range(nfb):
        r, cc = divmod(f, nhfb)
        D[8 * r:8 * r + 8, 8 * cc:8 * cc + 8] = np.asarray(d[f]).reshape(8, 8)
        V[8 * r:8 * r + 8, 8 * cc:8 * cc + 8] = np.asarray(v[f]).reshape(8, 8)
    dd = np.zeros((nfb, 16, 16), np.uint8)
    vv = np.zeros((nfb, 16, 16), np.int32)

    def fill(f, eh, ew):
        r, cc = divmod(f, nhfb)
        for by in range(eh):
            for bx in range(ew):
                y, x = 8 * r + by, 8 * cc + bx
                if y < nby and x < nbx and mask[y, x]:
                    dd[f, by, bx], vv[f, by, bx] = D[y, x], V[y, x]

    nb = 1 << prm.cdef_bits
    for f in range(nfb):
        if searched[f]:
            fill(f, 16 if kinds[f] in (1, 3) else 8, 16 if kinds[f] in (1, 2) else 8)
        elif applied and (ctl["ref_fs"] or kinds[f] < 0):
            si = int(fbs[f])
            ys, us = (int(prm.cdef_y_strength[si]), int(prm.cdef_uv_strength[si])) if si < nb else (0, 0)
            if ys or us:  # the apply filters this block: it finds the directions of its listed 8x8 blocks
                fill(f, 8, 8)
    return mse, skip, dd.reshape(nfb, 256), vv.reshape(nfb, 256)


def golden_cdef_tables(g, case):
    """The reference tables with the same zeroing (the reference leaves dir/var of skipped blocks untouched)."""
    c = pc.CASES[case]
    ctl = cdef_ctrl_row(c["cdef_level"])
    mse = np.array(g["cdef_mse"], np.uint64, copy=True)
    mse[:, :, ctl["n1"] + ctl["n2"]:] = 0
    return mse, g["cdef_skip"], g["cdef_dir"], g["cdef_var"]


# --------------------------------------------------------------------------- runners
def run_oracle(case):
    """The CPU restatement (oracle/) of the whole path."""
    import oracle
    c = pc.CASES[case]
    g = pc.load(case)
    src, rec, mi = pc.inputs(case)
    bd, w, h = c["bd"], c["w"], c["h"]
    dc = dlf_ctrls(c["dlf_level"])
    if dc["sb_based"]:  # LPF_PICK_FROM_Q levels (pinned on their own: test_dlf_byq) + the frame filter
        lfp = sb_dlf_params(c, [int(x) for x in g["lf_levels"]])
    else:
        lfp = oracle.dlf_pick(rec, src, bd, mi, pc.lf_params(c), dc["avg"], dc["avg_uv"], c["tl"], dc["early_exit"],
                              c["only4x4"])
    dlf = oracle.dlf_frame(rec, bd, mi, lfp)
    mask = pc.cdef_mask(mi)
    ctrls = oracle.controls(c["cdef_level"])
    ctrls.pred_y_f, ctrls.pred_uv_f = c["pred"]
    nvfb, nhfb = (((h + 7) & ~7) // 4 + 15) // 16, (((w + 7) & ~7) // 4 + 15) // 16
    fbb = np.ascontiguousarray(mi)["bsize"][::16, ::16].reshape(-1) if c["sb"] == 128 else None
    mse, skip, d, v = oracle.cdef_search_frame(dlf, src, bd, ctrls, c["q"], mask, fbb)
    kinds = oracle.cdef_fb_kinds(fbb, nvfb, nhfb) if fbb is not None else None
    prm, fbs = oracle.cdef_pick(w, h, mse, skip, ctrls, c["q"], int(g["cdef_lambda"][0]))
    if kinds is not None:
        fbs = oracle.cdef_dup_sb128(fbs, kinds, nvfb, nhfb)
    nb = 1 << prm.cdef_bits
    applied = int(prm.cdef_y_strength[0] != 0 or prm.cdef_uv_strength[0] != 0 or nb != 1)
    cdef = oracle.cdef_apply_frame(dlf, bd, mask, d, v, prm, fbs) if applied else [p.copy() for p in dlf]
    us = [c["us"][0], c["us"][1], c["us"][1]]
    lrc = oracle.lr_controls(c["wn_level"], c["sg_level"], c["rdmult"], c["sw"], c["wc"], c["sc"])
    ft, units, recs = oracle.lr_search_frame(cdef, src, bd, us, lrc)
    lr = oracle.lr_apply_frame(dlf, cdef, bd, ft, us, units) if any(ft) else [p.copy() for p in cdef]
    return dict(src=src, rec=rec, mi=mi, lf=lfp.levels(), dlf=dlf, tables=(mse, skip, d, v), prm=prm, nb=nb,
                fbs=fbs, applied=applied, cdef=cdef, ft=ft, units=units, recs=recs, lrc=lrc, lr=lr)


def run_gpu(case, ctx=None, async_=None):
    """The MI355X library (libsvtgpu) on the whole path, one stream, frames resident on the device.  async_ (default:
    SVTGPU_TEST_ASYNC=1 in the environment): the DLF level search and the LR search + RD finish in their asynchronous
    forms (svtgpu_dlf_pick_async + filter with the device levels, svtgpu_lr_search_frame_async + apply with the device
    units), the levels / frame types / units read back at the end."""
    import os
    if async_ is None:
        async_ = os.environ.get("SVTGPU_TEST_ASYNC") == "1"
    import svtgpu
    c = pc.CASES[case]
    g = pc.load(case)
    src, rec, mi = pc.inputs(case)
    bd, w, h = c["bd"], c["w"], c["h"]
    ctx = ctx or svtgpu.Context()
    S, R, D, C, O = (svtgpu.Frame(ctx, w, h, bd) for _ in range(5))
    S.upload(src)
    R.upload(rec)
    dl = svtgpu.DlfState(ctx, w, h)
    dl.set_mode_info(mi)
    if async_ and not dlf_ctrls(c["dlf_level"])["sb_based"]:
        dc = dlf_ctrls(c["dlf_level"])
        dl.pick_async(R, S, pc.lf_params(c), dc["avg"], dc["avg_uv"], c["tl"], dc["early_exit"], c["only4x4"])
        dl.filter_to(R, D, None)
        lfp = dl.read_levels()
    else:
        lfp = gpu_dlf_pick(dl, R, S, c)
        dl.filter_to(R, D, lfp)
    st = svtgpu.CdefState(ctx, w, h)
    st.set_block_mask(pc.cdef_mask(mi))
    if c["sb"] == 128:
        st.set_fb_bsize(np.ascontiguousarray(mi)["bsize"][::16, ::16].reshape(-1))
    ctrls = svtgpu.cdef_controls(c["cdef_level"])
    ctrls.pred_y_f, ctrls.pred_uv_f = c["pred"]
    st.search(D, S, ctrls, c["q"])
    tables = st.read()
    if async_:  # the pick in stream order; the apply reads its parameters on the device (zero strengths: a copy)
        st.pick_async(ctrls, c["q"], int(g["cdef_lambda"][0]))
        st.apply(D, C, None)
    else:
        prm, fbs = st.pick(ctrls, c["q"], int(g["cdef_lambda"][0]))
        nb = 1 << prm.cdef_bits
        applied = int(prm.cdef_y_strength[0] != 0 or prm.cdef_uv_strength[0] != 0 or nb != 1)
        if applied:
            st.apply(D, C, prm)
        else:
            svtgpu.check(svtgpu.lib().svtgpu_frame_copy(C.h, D.h, None))
    us = [c["us"][0], c["us"][1], c["us"][1]]
    lr = svtgpu.LrState(ctx, w, h, us)
    lrc = svtgpu.lr_controls(c["wn_level"], c["sg_level"], c["rdmult"], c["sw"], c["wc"], c["sc"])
    if async_:
        lr.search_async(C, S, lrc)
        lr.apply(D, C, O, None)
        ft, recs = lr.read_result(), None
        units = [lr.read_units(p) for p in range(3)]
    else:
        ft, recs = lr.search(C, S, lrc, records=True)
        units = svtgpu.lr_finish_frame(lrc, recs)[1]
        if any(ft):
            lr.apply(D, C, O, ft)
        else:
            svtgpu.check(svtgpu.lib().svtgpu_frame_copy(O.h, C.h, None))
    ctx.synchronize()
    if async_:
        prm, fbs = st.read_params()
        nb = 1 << prm.cdef_bits
        applied = int(prm.cdef_y_strength[0] != 0 or prm.cdef_uv_strength[0] != 0 or nb != 1)
    out = dict(src=src, rec=rec, mi=mi, lf=lfp.levels(), dlf=D.download(), tables=tables, prm=prm, nb=nb, fbs=fbs,
               applied=applied, cdef=C.download(), ft=ft, units=units, recs=recs, lrc=lrc, lr=O.download())
    for x in (S, R, D, C, O, dl, st, lr):
        x.close()
    return out


# --------------------------------------------------------------------------- comparison
def _planes_equal(g, key, got, digest, what):
    for p in range(3):
        a = np.ascontiguousarray(got[p], np.uint16)
        if digest:
            assert pc.digest(a) == str(g["sha_%s%d" % (key, p)]), "%s: %s plane %d differs (digest)" % (what, key, p)
        else:
            np.testing.assert_array_equal(a, g["%s%d" % (key, p)], err_msg="%s: %s plane %d" % (what, key, p))


def check(case, out, what):
    """Assert `out` (run_gpu / run_oracle) equals the reference outputs of `case`, stage by stage."""
    c = pc.CASES[case]
    g = pc.load(case)
    digest = c["digest"]
    assert pc.input_digest(out["src"], out["rec"], out["mi"]) == str(g["input_sha"]), \
        "%s: input generator differs from the fixture's" % case
    # DLF
    assert tuple(int(x) for x in out["lf"]) == tuple(int(x) for x in g["lf_levels"]), (what, case, out["lf"],
                                                                                      g["lf_levels"])
    _planes_equal(g, "dlf", out["dlf"], digest, what + " " + case)
    # CDEF search tables (in the reference's layout) and the picked strengths
    mse, skip, dd, vv = reference_layout(case, out["mi"], *out["tables"], out["fbs"], out["prm"], out["applied"])
    names = ("cdef_mse", "cdef_skip", "cdef_dir", "cdef_var")
    if digest:
        for k, a in zip(names, (mse, skip, dd, vv)):
            ref = g.get("sha_" + k)
            if ref is not None:
                assert pc.digest(a) == str(ref), "%s %s: %s differs (digest)" % (what, case, k)
            else:
                np.testing.assert_array_equal(a, g[k], err_msg="%s %s %s" % (what, case, k))
    else:
        gm, gs, gd, gv = golden_cdef_tables(g, case)
        np.testing.assert_array_equal(skip, gs, err_msg="%s %s cdef_skip" % (what, case))
        np.testing.assert_array_equal(mse, gm, err_msg="%s %s cdef_mse" % (what, case))
        np.testing.assert_array_equal(dd, gd, err_msg="%s %s cdef_dir" % (what, case))
        np.testing.assert_array_equal(vv, gv, err_msg="%s %s cdef_var" % (what, case))
    prm = out["prm"]
    gp = [int(x) for x in g["cdef_params"]]
    nb = out["nb"]
    got = [prm.cdef_damping, prm.cdef_bits, nb, out["applied"]] + \
        [int(prm.cdef_y_strength[k]) if k < nb else gp[4 + k] for k in range(8)] + \
        [int(prm.cdef_uv_strength[k]) if k < nb else gp[12 + k] for k in range(8)]
    assert got == gp, (what, case, got, gp)
    np.testing.assert_array_equal(np.asarray(out["fbs"], np.int8), g["cdef_fbs"],
                                  err_msg="%s %s cdef_fbs" % (what, case))
    _planes_equal(g, "cdef", out["cdef"], digest, what + " " + case)
    # LR
    assert [int(x) for x in out["ft"]] == [int(x) for x in g["lr_ftype"]], (what, case, out["ft"], g["lr_ftype"])
    import lr_cases
    import svtgpu
    ref = dict(name="%s %s" % (what, case), ftype=[int(x) for x in g["lr_ftype"]], ctrls=out["lrc"],
               units=[svtgpu.rest_units_from_rows(g["lr_units%d" % p]) for p in range(3)],
               sse=[g["lr_sse%d" % p] for p in range(3)], rec_params=[g["lr_rec%d" % p] for p in range(3)])
    lr_cases.compare_search(out["ft"], out["units"], out["recs"], ref)
    _planes_equal(g, "lr", out["lr"], digest, what + " " + case)


# --------------------------------------------------------------------------- one rank of a picture tiled over GPUs
def run_gpu_tiled(case, rank, world, comm, ctx=None):
    """This rank's part of `case` with the picture tiled over `world` ranks (svtgpu_tile_plan, 1 x 2 / 2 x 2 / 2 x 4
    grids): the frame-level calls exchange the DLF trial SSEs, the CDEF search tables and the LR search records over
    `comm` (svtgpu.Comm).  Returns the rank's crops (the DLF output over its tile, the CDEF and LR outputs over its
    LR units) plus the frame-level decisions every rank takes; assemble_tiled() puts the ranks' parts together."""
    import svtgpu
    c = pc.CASES[case]
    g = pc.load(case)
    src, rec, mi = pc.inputs(case)
    bd, w, h = c["bd"], c["w"], c["h"]
    us = [c["us"][0], c["us"][1], c["us"][1]]
    gx, gy = svtgpu.tile_grid(world)
    plan = svtgpu.tile_plan(w, h, us, gx, gy, rank, sb=c["sb"]).rects()
    ctx = ctx or svtgpu.Context()
    S, R, D, C, O = (svtgpu.Frame(ctx, w, h, bd) for _ in range(5))
    # the rank's inputs: only the plan's in_rect of the recon and the source, the rest of both pictures poisoned (a
    # read outside in_rect changes the outputs, which are checked against the reference's)
    rng = np.random.default_rng(7 + rank)
    for F in (S, R):
        F.upload([rng.integers(0, 1 << bd, size=F.plane_shape(p), dtype=np.uint16) for p in range(3)])
    S.upload(src, rect=plan["in_rect"])
    R.upload(rec, rect=plan["in_rect"])
    dl = svtgpu.DlfState(ctx, w, h)
    dl.set_mode_info(mi)
    dl.set_tile(plan["tile"], plan["dlf_out"], comm)
    lfp = gpu_dlf_pick(dl, R, S, c)
    dl.filter_to(R, D, lfp)
    st = svtgpu.CdefState(ctx, w, h)
    st.set_block_mask(pc.cdef_mask(mi))
    if c["sb"] == 128:
        st.set_fb_bsize(np.ascontiguousarray(mi)["bsize"][::16, ::16].reshape(-1))
    st.set_tile(plan["fb_rect"], plan["cdef_out"], comm)
    ctrls = svtgpu.cdef_controls(c["cdef_level"])
    ctrls.pred_y_f, ctrls.pred_uv_f = c["pred"]
    st.search(D, S, ctrls, c["q"])
    prm, fbs = st.pick(ctrls, c["q"], int(g["cdef_lambda"][0]))
    tables = st.read()  # after the pick: every rank's blocks, summed over the ranks
    nb = 1 << prm.cdef_bits
    applied = int(prm.cdef_y_strength[0] != 0 or prm.cdef_uv_strength[0] != 0 or nb != 1)
    if applied:
        st.apply(D, C, prm)
    else:
        svtgpu.check(svtgpu.lib().svtgpu_frame_copy(C.h, D.h, None))
    lr = svtgpu.LrState(ctx, w, h, us)
    lr.set_tile(plan["lr_units"], plan["lr_out"], comm)
    lrc = svtgpu.lr_controls(c["wn_level"], c["sg_level"], c["rdmult"], c["sw"], c["wc"], c["sc"])
    ft, recs = lr.search(C, S, lrc, records=True)
    units = svtgpu.lr_finish_frame(lrc, recs)[1]
    if any(ft):
        lr.apply(D, C, O, ft)
    else:
        svtgpu.check(svtgpu.lib().svtgpu_frame_copy(O.h, C.h, None))
    ctx.synchronize()

    def crop(planes, rects):
        return [np.ascontiguousarray(planes[p][r[1]:r[3], r[0]:r[2]]) for p, r in enumerate(rects)]
    t = plan["tile"]
    tile3 = [t, [t[0] // 2, t[1] // 2, t[2] // 2, t[3] // 2], [t[0] // 2, t[1] // 2, t[2] // 2, t[3] // 2]]
    out = dict(rank=rank, plan=plan, tile3=tile3, lf=lfp.levels(), dlf=crop(D.download(), tile3), tables=tables,
               prm=prm.as_tuple(), nb=nb, fbs=fbs, applied=applied, cdef=crop(C.download(), plan["lr_out"]), ft=ft,
               units=units, recs=recs, lr=crop(O.download(), plan["lr_out"]))
    for x in (S, R, D, C, O, dl, st, lr):
        x.close()
    return out


def assemble_tiled(case, parts):
    """The ranks' parts of run_gpu_tiled as one run_gpu-style result (frame-level decisions must agree)."""
    import svtgpu
    c = pc.CASES[case]
    src, rec, mi = pc.inputs(case)
    w, h = c["w"], c["h"]
    p0 = parts[0]
    for q in parts[1:]:
        assert tuple(q["lf"]) == tuple(p0["lf"]) and q["prm"] == p0["prm"] and list(q["ft"]) == list(p0["ft"])
        assert np.array_equal(q["fbs"], p0["fbs"])
        for a, b in zip(q["tables"], p0["tables"]):
            assert np.array_equal(a, b)
        for p in range(3):
            assert q["recs"][p].tobytes() == p0["recs"][p].tobytes()
    shapes = [(h, w), (h // 2, w // 2), (h // 2, w // 2)]
    full = {k: [np.zeros(s, np.uint16) - 1 for s in shapes] for k in ("dlf", "cdef", "lr")}
    for q in parts:
        for key, rects in (("dlf", q["tile3"]), ("cdef", q["plan"]["lr_out"]), ("lr", q["plan"]["lr_out"])):
            for p, r in enumerate(rects):
                full[key][p][r[1]:r[3], r[0]:r[2]] = q[key][p]
    prm = svtgpu.CdefParams()
    prm.cdef_damping, prm.cdef_bits = p0["prm"][0], p0["prm"][1]
    for k, (y, uv) in enumerate(zip(p0["prm"][2], p0["prm"][3])):
        prm.cdef_y_strength[k], prm.cdef_uv_strength[k] = y, uv
    lrc = svtgpu.lr_controls(c["wn_level"], c["sg_level"], c["rdmult"], c["sw"], c["wc"], c["sc"])
    return dict(src=src, rec=rec, mi=mi, lf=p0["lf"], dlf=full["dlf"], tables=p0["tables"], prm=prm, nb=p0["nb"],
                fbs=p0["fbs"], applied=p0["applied"], cdef=full["cdef"], ft=p0["ft"], units=p0["units"],
                recs=p0["recs"], lrc=lrc, lr=full["lr"])


# --------------------------------------------------------------------------- a picture off the 8-sample grid, tiled
def run_crop(c, crop, rank=0, world=1, comm=None, ctx=None, lam=60000):
    """The whole path on a synthetic case dict `c` (pipeline_cases._case: w x h the 8-aligned coded size) whose crop
    size `crop` = (w, h) is below it: the DLF state told the crop (svtgpu_dlf_set_crop), the CDEF on the coded frames,
    the LR state at the crop size.  world > 1: this rank's part of the picture tiled with svtgpu_tile_plan_crop (the
    rest of its input pictures poisoned).  Returns the decisions and the output planes (whole frames; a rank's are
    valid inside its plan's rects)."""
    import svtgpu
    bd, w, h = c["bd"], c["w"], c["h"]
    src, rec = pc.frame_pair(w, h, bd, c["seed"])
    mi = pc.mode_info(c)
    us = [c["us"][0], c["us"][1], c["us"][1]]
    ctx = ctx or svtgpu.Context()
    S, R, D, C, O = (svtgpu.Frame(ctx, w, h, bd) for _ in range(5))
    plan = None
    if world > 1:
        plan = svtgpu.tile_plan(w, h, us, *svtgpu.tile_grid(world), rank, sb=c["sb"], crop=crop).rects()
        rng = np.random.default_rng(17 + rank)
        for F in (S, R):
            F.upload([rng.integers(0, 1 << bd, size=F.plane_shape(p), dtype=np.uint16) for p in range(3)])
        S.upload(src, rect=plan["in_rect"])
        R.upload(rec, rect=plan["in_rect"])
    else:
        S.upload(src)
        R.upload(rec)
    dl = svtgpu.DlfState(ctx, w, h)
    dl.set_crop(*crop)
    dl.set_mode_info(mi)
    if plan:
        dl.set_tile(plan["tile"], plan["dlf_out"], comm)
    lfp = gpu_dlf_pick(dl, R, S, c)
    dl.filter_to(R, D, lfp)
    st = svtgpu.CdefState(ctx, w, h)
    st.set_block_mask(pc.cdef_mask(mi))
    if plan:
        st.set_tile(plan["fb_rect"], plan["cdef_out"], comm)
    ctrls = svtgpu.cdef_controls(c["cdef_level"])
    st.search(D, S, ctrls, c["q"])
    prm, fbs = st.pick(ctrls, c["q"], lam)
    st.apply(D, C, prm)
    lr = svtgpu.LrState(ctx, crop[0], crop[1], us)
    if plan:
        lr.set_tile(plan["lr_units"], plan["lr_out"], comm)
    lrc = svtgpu.lr_controls(c["wn_level"], c["sg_level"], c["rdmult"], c["sw"], c["wc"], c["sc"])
    ft, recs = lr.search(C, S, lrc, records=True)
    lr.apply(D, C, O, ft)
    ctx.synchronize()
    out = dict(plan=plan, lf=tuple(lfp.levels()), prm=prm.as_tuple(), fbs=fbs, ft=list(ft), recs=recs,
               dlf=D.download(), cdef=C.download(), lr=O.download())
    for x in (S, R, D, C, O, dl, st, lr):
        x.close()
    return out


def compare_crop_parts(single, parts):
    """Every rank's decisions equal the single-GPU run's, and its outputs inside its plan's rects (the DLF output over
    its tile, the CDEF and LR outputs over its LR units' samples) equal the single-GPU planes."""
    for q in parts:
        assert q["lf"] == single["lf"] and q["prm"] == single["prm"] and q["ft"] == single["ft"], (q["lf"], single["lf"])
        assert np.array_equal(q["fbs"], single["fbs"])
        for p in range(3):
            assert q["recs"][p].tobytes() == single["recs"][p].tobytes(), p
        t = q["plan"]["tile"]
        tile3 = [t] + [[t[0] // 2, t[1] // 2, (t[2] + 1) // 2, (t[3] + 1) // 2]] * 2
        for key, rects in (("dlf", tile3), ("cdef", q["plan"]["lr_out"]), ("lr", q["plan"]["lr_out"])):
            for p, r in enumerate(rects):
                a = q[key][p][r[1]:r[3], r[0]:r[2]]
                b = single[key][p][r[1]:r[3], r[0]:r[2]]
                assert np.array_equal(a, b), (key, p, r)
