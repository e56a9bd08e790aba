"""Frame-buffer work around the path on the MI355X: the RTCD shims against the reference's goldens
(tests/golden/frame_ops.bin), the device-pointer kernels at 4K against the CPU oracle, and svtgpu_frame_convert round
trips.  Bit-exact."""
import ctypes

import numpy as np
import pytest

import frame_cases as fc
import oracle
import svtgpu

pytestmark = pytest.mark.gpu
P = lambda a: ctypes.c_void_p(a.ctypes.data)


@pytest.fixture(scope="module")
def g():
    return fc.golden()


def test_convert_shims_golden(g):
    L = svtgpu.lib()
    for src, d0, d1, w, h, ss, ds in fc.conv_cases(g):
        d = d0.copy()
        if src.dtype == np.uint8:
            L.svtgpu_convert_8bit_to_16bit(P(src), ss, P(d), ds, w, h)
        else:
            L.svtgpu_convert_16bit_to_8bit(P(src), ss, P(d), ds, w, h)
        np.testing.assert_array_equal(d, d1, err_msg="%dx%d" % (w, h))


def test_padding_shims_golden(g):
    L = svtgpu.lib()
    for b0, b1, w, h, st, pw, ph in fc.pad_cases(g):
        b = b0.copy()
        if b.dtype == np.uint8:
            L.svtgpu_aom_generate_padding(P(b), st, w, h, pw, ph)
        else:
            L.svtgpu_aom_generate_padding16_bit(P(b), st, w, h, pw, ph)
        np.testing.assert_array_equal(b, b1, err_msg="%dx%d pad %d,%d" % (w, h, pw, ph))


def test_extend_shim_golden(g):
    L = svtgpu.lib()
    for b0, b1, w, h, st, bh, bv, off in fc.ext_cases(g):
        b = b0.copy()
        if b.dtype == np.uint8:
            L.svtgpu_extend_frame(ctypes.c_void_p(b.ctypes.data + off), w, h, st, bh, bv, 0)
        else:  # CONVERT_TO_BYTEPTR
            L.svtgpu_extend_frame(ctypes.c_void_p((b.ctypes.data + 2 * off) >> 1), w, h, st, bh, bv, 1)
        np.testing.assert_array_equal(b, b1, err_msg="%dx%d ext %d,%d" % (w, h, bh, bv))


def test_device_kernels_4k_vs_oracle():
    """3840x2160 planes through the device-pointer entry points (the frame sizes the encoder runs them at): conversion
    both ways, reference padding of a 10-bit plane with an 80-sample border, extension of an 8-bit plane."""
    import torch
    L = svtgpu.lib()
    svtgpu.Context(0)
    rng = np.random.default_rng(11)
    W, H = 3840, 2160
    src8 = rng.integers(0, 256, size=(H, W), dtype=np.uint8)
    d16 = torch.zeros((H, W + 64), dtype=torch.int16, device="cuda")
    s8 = torch.from_numpy(src8).cuda()
    torch.cuda.synchronize()  # the library runs on its own stream
    assert L.svtgpu_convert_plane(ctypes.c_void_p(s8.data_ptr()), 8, W, ctypes.c_void_p(d16.data_ptr()), 16, W + 64, W,
                                  H, None) == 0
    torch.cuda.synchronize()
    out16 = d16.cpu().numpy().view(np.uint16)
    want = np.zeros((H, W + 64), np.uint16)
    oracle.convert(src8.ravel(), W, want.ravel(), W + 64, W, H)
    np.testing.assert_array_equal(out16, want)
    back = torch.zeros((H, W), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()  # the fill runs on torch's stream, the conversion on the library's
    assert L.svtgpu_convert_plane(ctypes.c_void_p(d16.data_ptr()), 16, W + 64, ctypes.c_void_p(back.data_ptr()), 8, W,
                                  W, H, None) == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(back.cpu().numpy(), src8)
    # padding: 10-bit plane, 80-sample border, stride with slack
    pw = ph = 80
    st = W + 2 * pw + 32
    buf = rng.integers(0, 1024, size=(H + 2 * ph) * st, dtype=np.uint16)
    dbuf = torch.from_numpy(buf.view(np.int16).copy()).cuda()
    torch.cuda.synchronize()
    assert L.svtgpu_pad_plane(ctypes.c_void_p(dbuf.data_ptr()), 16, st, W, H, pw, ph, None) == 0
    torch.cuda.synchronize()
    want = buf.copy()
    oracle.pad(want, st, W, H, pw, ph)
    np.testing.assert_array_equal(dbuf.cpu().numpy().view(np.uint16), want)
    # extension: 8-bit plane, 32 x 16 border
    bh, bv = 32, 16
    st = W + 2 * bh + 8
    buf8 = rng.integers(0, 256, size=(H + 2 * bv) * st, dtype=np.uint8)
    off = bv * st + bh
    dbuf8 = torch.from_numpy(buf8.copy()).cuda()
    torch.cuda.synchronize()
    assert L.svtgpu_extend_plane(ctypes.c_void_p(dbuf8.data_ptr() + off), 8, st, W, H, bh, bv, None) == 0
    torch.cuda.synchronize()
    want8 = buf8.copy()
    oracle.extend(want8, off, st, W, H, bh, bv)
    np.testing.assert_array_equal(dbuf8.cpu().numpy(), want8)


def test_frame_convert_round_trip():
    """svt_convert_pic_8bit_to_16bit then the 16 -> 8 copy-back: identity on 8-bit content, every plane."""
    import synth
    ctx = svtgpu.Context(0)
    W, H = 1920, 1080
    src, _ = synth.frame_pair(W, H, 8, seed=0x5EED0021)
    f8, f16, g8 = svtgpu.Frame(ctx, W, H, 8), svtgpu.Frame(ctx, W, H, 10), svtgpu.Frame(ctx, W, H, 8)
    f8.upload(src)
    assert svtgpu.lib().svtgpu_frame_convert(f8.h, f16.h, None) == 0
    up = f16.download()
    assert all(np.array_equal(a.astype(np.uint16), b) for a, b in zip(src, up))
    assert svtgpu.lib().svtgpu_frame_convert(f16.h, g8.h, None) == 0
    assert all(np.array_equal(a, b) for a, b in zip(src, g8.download()))
