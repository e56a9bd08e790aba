"""libsvtgpu inside the reference encoder: the drop-in proof.

oracle/enc.mk builds the reference's own encoder library (every C source of Source/Lib/{Common,Encoder}, C-only) and
oracle/ref_harness/enc_drop_in.c drives it through its public API (svt_av1_enc_init_handle / _set_parameter / _init /
_send_picture / _get_packet) over a synthetic 10-bit 4:2:0 clip with deblocking, CDEF and loop restoration (Wiener +
self-guided, preset 2) on.  The bitstream with include/svtgpu_rtcd.h's svtgpu_install_filter_rtcd() called after
svt_av1_enc_init (the encoder's own process bodies then run libsvtgpu's device kernels through its RTCD pointers)
must equal the bitstream of the encoder as built, byte for byte; so must the bitstream with the frame-level hooks
(oracle/ref_harness/enc_frame_hooks.c: the encoder's own DLF / CDEF / LR process bodies call svtgpu_dlf_pick /
svtgpu_dlf_frame, svtgpu_cdef_search_frame / _pick / _apply_frame and svtgpu_lr_search_frame / _finish_plane /
_apply_frame in place of their frame-level C functions, bound by ELF symbol interposition).  Test infrastructure: the reference build lives in
oracle/_ref (git-ignored; built here by __graft_entry__.build(), shipped to the GPU box with the tree)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_ref", "enc", "enc_drop_in")

needs_exe = pytest.mark.skipif(not os.path.exists(EXE), reason="oracle/_ref/enc not built (needs /root/reference)")


# the encoder with the CDEF process body's per-segment CPU search removed (oracle/ref_harness/no_seg_search.py: a /tmp
# copy of EbCdefProcess.c with its one cdef_seg_search call taken out; INTEGRATION.md §2 applied)
EXE_NSS = os.path.join(ROOT, "oracle", "_ref", "enc", "nss", "enc_drop_in")
OBJ = os.path.join(ROOT, "oracle", "_ref", "enc", "obj", "Source", "Lib", "Encoder", "Codec", "EbCdefProcess.o")
OBJ_NSS = os.path.join(ROOT, "oracle", "_ref", "enc", "nss", "EbCdefProcess.o")
# the encoder with the fork's CCSO search / apply switched back on (oracle/ref_harness/with_ccso.py)
EXE_CCSO = os.path.join(ROOT, "oracle", "_ref", "enc", "ccso", "enc_drop_in")
needs_ccso = pytest.mark.skipif(not os.path.exists(EXE_CCSO), reason="oracle/_ref/enc/ccso not built (needs /root/reference)")


def _encode(mode, path, *args, timeout=600, exe=EXE):
    r = subprocess.run([exe, mode, path] + [str(a) for a in args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (mode, r.returncode, r.stderr[-2000:])
    out = {}
    for l in r.stdout.splitlines():  # "<mode> bytes <n> packets <n> ..." and (frame mode) "frame kinds <k> <n> ..."
        f = l.split()
        if f[:2] == [mode, "bytes"] or f[:2] == ["frame", "kinds"]:
            start = 1 if f[1] == "bytes" else 2
            out.update({f[i]: int(f[i + 1]) for i in range(start, len(f) - 1, 2)})
    return out


@needs_exe
def test_reference_encoder_runs_cpu(tmp_path):
    """The reference encoder as built encodes the clip deterministically (two runs, same bytes)."""
    a, b = str(tmp_path / "a.obu"), str(tmp_path / "b.obu")
    ia, ib = _encode("cpu", a, 160, 128, 3, 2, 40), _encode("cpu", b, 160, 128, 3, 2, 40)
    assert ia["bytes"] > 0 and ia["packets"] >= 3
    assert open(a, "rb").read() == open(b, "rb").read()


@needs_exe
@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("geom", [(320, 192, 5, 2, 40), (256, 144, 3, 2, 20)])
def test_encoder_bitstream_identical_with_filter_rtcd(tmp_path, geom):
    """The reference encoder with libsvtgpu's filter RTCD shims installed (svtgpu_install_filter_rtcd after
    svt_av1_enc_init) writes the same bitstream as without them; the shims really ran (svtgpu_shim_calls)."""
    cpu, gpu = str(tmp_path / "cpu.obu"), str(tmp_path / "gpu.obu")
    ic = _encode("cpu", cpu, *geom)
    ig = _encode("rtcd", gpu, *geom)
    assert ig["shim_calls"] > 1000, ig
    assert ic["bytes"] == ig["bytes"] and open(cpu, "rb").read() == open(gpu, "rb").read(), (ic, ig)


@needs_exe
@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("geom", [(320, 192, 5, 2, 40), (256, 144, 3, 2, 20), (384, 256, 4, 1, 32),
                                  (250, 138, 3, 2, 40)])
def test_encoder_bitstream_identical_with_frame_hooks(tmp_path, geom):
    """The encoder's DLF / CDEF / LR process bodies calling libsvtgpu's frame-level API (level searches, strength
    pick, restoration search + RD finish, the three frame filters on the device) write the same bitstream as the
    encoder as built; every hooked call was served by the device path (no fallback).  250 x 138: a picture off the
    8-sample grid (the encoder pads it to 256 x 144; loop restoration covers the 250 x 138 crop, chroma 125 x 69)."""
    cpu, gpu = str(tmp_path / "cpu.obu"), str(tmp_path / "frame.obu")
    ic = _encode("cpu", cpu, *geom)
    ig = _encode("frame", gpu, *geom)
    assert ig["frame_calls"] >= 3 * geom[2] and ig["frame_fallbacks"] == 0, ig
    # every stage ran on the device for every frame, and restoration really filtered some frames
    for k in ("dlf_pick", "dlf_frame", "cdef_pick", "lr_search"):
        assert ig[k] >= geom[2], (k, ig)
    assert ig["cdef_apply"] >= 1 and ig["lr_apply"] >= 1 and ig["lr_on"] >= 1, ig
    assert ic["bytes"] == ig["bytes"] and open(cpu, "rb").read() == open(gpu, "rb").read(), (ic, ig)


# Round 6: the configurations an encoder actually runs.  args: width height frames preset qp
# bit_depth logical_processors.  Presets 3 and 4 run Wiener level 5 (luma only, non-last layers) beside self-guided
# level 3 (luma and chroma, ep_inc 8): rest_finish_search's switchable pass over a chroma plane then reads luma's entries
# of the shared RestUnitSearchInfo array (svtgpu_lr_finish_frame; the device finish models the same).  8-bit: the
# encoder's 8-bit pipeline (is_16bit_pipeline = 0, EbEncHandle.c:4534) through the hooks' 8-bit branch.  Four logical
# processors: several pictures through the DLF / CDEF / REST processes -- and the hooks' per-picture device state -- at
# once.  640 x 360: a larger picture (more units per plane, SB rows of every kind).
WIDE = [
    ("preset3", (320, 192, 5, 3, 40, 10, 1)),
    ("preset4", (320, 192, 5, 4, 44, 10, 1)),
    ("8bit_p2", (320, 192, 4, 2, 40, 8, 1)),
    ("8bit_p3", (256, 144, 4, 3, 36, 8, 1)),
    ("lp4_p2", (320, 192, 6, 2, 40, 10, 4)),
    ("640x360_p3", (640, 360, 3, 3, 40, 10, 2)),
]


@needs_exe
@pytest.mark.gpu
@pytest.mark.timeout(1200)
@pytest.mark.parametrize("name,geom", WIDE)
def test_encoder_bitstream_identical_wide(tmp_path, name, geom):
    """Frame-level hooks and the filter RTCD shims, each against the encoder as built, byte for byte, with every hooked
    call served by the device."""
    cpu, frm, rt = str(tmp_path / "cpu.obu"), str(tmp_path / "frame.obu"), str(tmp_path / "rtcd.obu")
    ic = _encode("cpu", cpu, *geom, timeout=1100)
    ig = _encode("frame", frm, *geom, timeout=1100)
    assert ig["frame_fallbacks"] == 0 and ig["frame_calls"] >= 3 * geom[2], (name, ig)
    for k in ("dlf_pick", "dlf_frame", "cdef_pick"):
        assert ig[k] >= geom[2], (name, k, ig)
    assert ic["bytes"] == ig["bytes"] and open(cpu, "rb").read() == open(frm, "rb").read(), (name, ic, ig)
    # restoration is per picture (EncModeConfig.c:1884-1903: the Wiener level depends on is_not_last_layer), and at
    # preset 4 some pictures have it off, so the search runs on a subset of the frames -- at least one.  Preset 4's
    # luma-only Wiener level 5 picks RESTORE_NONE for every unit of this clip (the RD finish still runs on the device
    # and must agree); the other cases really filter
    assert ig["lr_search"] >= 1, (name, ig)
    assert name == "preset4" or ig["lr_on"] >= 1, (name, ig)
    ir = _encode("rtcd", rt, *geom, timeout=1100)
    assert ir["shim_calls"] > 1000, (name, ir)
    assert open(cpu, "rb").read() == open(rt, "rb").read(), (name, ic, ir)


@pytest.mark.skipif(not os.path.exists(OBJ_NSS), reason="oracle/_ref/enc/nss not built (needs /root/reference)")
def test_no_seg_search_build_drops_the_cpu_search():
    """The edited CDEF process body no longer contains the per-segment search: the static cdef_seg_search is defined
    in the encoder's own object and absent from the edited one (unreferenced after the edit, the compiler drops it),
    and the edited object references no other symbol than the original does."""
    def syms(path):
        r = subprocess.run(["nm", path], capture_output=True, text=True, check=True)
        return {l.split()[-1]: l.split()[-2] for l in r.stdout.splitlines() if l.strip()}
    a, b = syms(OBJ), syms(OBJ_NSS)
    assert "cdef_seg_search" in a and "cdef_seg_search" not in b
    assert {k for k, t in b.items() if t == "U"} <= {k for k, t in a.items() if t == "U"} | {"svt_aom_assert_err"}


@pytest.mark.skipif(not os.path.exists(EXE_NSS), reason="oracle/_ref/enc/nss not built (needs /root/reference)")
@pytest.mark.gpu
@pytest.mark.timeout(1200)
@pytest.mark.parametrize("name,geom", [("p2_10bit", (320, 192, 5, 2, 40, 10, 1)), ("8bit_p3", (256, 144, 4, 3, 36, 8, 1)),
                                       ("640x360_p3_lp2", (640, 360, 3, 3, 40, 10, 2))])
def test_encoder_without_cpu_cdef_search(tmp_path, name, geom):
    """The encoder with the per-segment CPU search removed from its CDEF process body and finish_cdef_search /
    svt_av1_cdef_frame (and the DLF / LR frame functions) served by the device writes the bitstream of the encoder as
    built, byte for byte, every hooked call on the device: nothing of the CPU search's output was needed."""
    cpu, frm = str(tmp_path / "cpu.obu"), str(tmp_path / "frame_nss.obu")
    ic = _encode("cpu", cpu, *geom, timeout=1100)
    ig = _encode("frame", frm, *geom, timeout=1100, exe=EXE_NSS)
    assert ig["frame_fallbacks"] == 0 and ig["cdef_pick"] >= geom[2], (name, ig)
    assert ic["bytes"] == ig["bytes"] and open(cpu, "rb").read() == open(frm, "rb").read(), (name, ic, ig)


@needs_ccso
def test_ccso_build_runs_ccso(tmp_path):
    """The encoder with its CCSO calls switched back on (EbCdefProcess.c:621-623) encodes deterministically and writes a
    different bitstream from the encoder as shipped: the CCSO frame header and block flags are coded and its filtering
    feeds later pictures' prediction -- so an equal bitstream below is a check of the CCSO decisions and samples."""
    a, b, c = str(tmp_path / "a.obu"), str(tmp_path / "b.obu"), str(tmp_path / "c.obu")
    geom = (384, 256, 3, 2, 40, 8, 1)
    ia, ib = _encode("cpu", a, *geom, exe=EXE_CCSO), _encode("cpu", b, *geom, exe=EXE_CCSO)
    _encode("cpu", c, *geom)
    assert ia["bytes"] > 0 and open(a, "rb").read() == open(b, "rb").read()
    assert open(a, "rb").read() != open(c, "rb").read()


@needs_ccso
@pytest.mark.gpu
@pytest.mark.timeout(1200)
@pytest.mark.parametrize("name,geom", [("384x256_p2", (384, 256, 3, 2, 40, 8, 1)),
                                       ("520x296_p3", (520, 296, 4, 3, 36, 8, 1))])
def test_encoder_with_ccso_on_device(tmp_path, name, geom):
    """The CCSO-enabled encoder with ccso_search / ccso_frame (and the DLF / CDEF / LR frame functions) served by the
    device writes the bitstream of the same encoder on the CPU, byte for byte: the frame header's CCSO fields, the
    per-block flags and the filtered recon all equal the fork's own C.  Every CCSO call on the device (no fallback)
    and some plane enabled.  One logical processor: the fork's CPU search keeps its state in file-scope globals
    (EbPickccso.c:18-41), so two pictures searching at once crash the reference itself (seen at lp 2)."""
    cpu, frm = str(tmp_path / "cpu.obu"), str(tmp_path / "frame.obu")
    ic = _encode("cpu", cpu, *geom, timeout=1100, exe=EXE_CCSO)
    ig = _encode("frame", frm, *geom, timeout=1100, exe=EXE_CCSO)
    assert ig["frame_fallbacks"] == 0, (name, ig)
    assert ig["ccso_search"] >= geom[2] and ig["ccso_apply"] >= geom[2] and ig["ccso_on"] >= 1, (name, ig)
    assert ic["bytes"] == ig["bytes"] and open(cpu, "rb").read() == open(frm, "rb").read(), (name, ic, ig)
