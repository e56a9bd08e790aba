"""Reader for the golden-vector container written by oracle/ref_harness/golden_io.h."""
import struct

import numpy as np

_DT = {"B": np.uint8, "b": np.int8, "H": np.uint16, "h": np.int16, "I": np.uint32,
       "i": np.int32, "Q": np.uint64, "q": np.int64, "d": np.float64}


def load(path):
    out = {}
    with open(path, "rb") as f:
        data = f.read()
    assert data[:4] == b"SVTG", path
    off = 8
    while off < len(data):
        (nl,) = struct.unpack_from("<H", data, off)
        off += 2
        name = data[off:off + nl].decode()
        off += nl
        dt, nd = struct.unpack_from("<cB", data, off)
        off += 2
        dims = struct.unpack_from("<%dI" % nd, data, off)
        off += 4 * nd
        dtype = np.dtype(_DT[dt.decode()])
        n = int(np.prod(dims)) if dims else 1
        # a copy: records start at arbitrary byte offsets, and the highbd shims take CONVERT_TO_BYTEPTR pointers
        # (address >> 1), which need 2-byte aligned uint16 data
        arr = np.frombuffer(data, dtype=dtype, count=n, offset=off).reshape(dims).copy()
        off += n * dtype.itemsize
        out[name] = arr
    return out
