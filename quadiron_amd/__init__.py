"""quadiron_amd -- MI355X-native RS-FNT erasure coding (Reed-Solomon over
GF(65537) via the Fermat Number Transform), a drop-in for QuadIron's RS-FNT
path.

The product is the native library ``quadiron_amd/libquadiron_amd.so`` (HIP
kernels for gfx950 + C++ host layer) exporting:

* the drop-in C-ABI ``quadiron_fnt32_*`` (include/quadiron_c.h),
* the device-level C-ABI ``qi_plan_* / qi_gpu_*`` (include/qi_gpu.h),
* the C view of the block API ``qi_fec_*`` (include/qi_gpu.h).

This module only loads it with ctypes and wraps those entry points for
Python callers (tests, bench).  There is no Python or CPU compute path: if
the library or a HIP device is missing, calls fail loudly.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# QI_LIB_PATH: load another build of the same library (A/B timing of kernel
# variants built by tools/ab_build.sh); the default is the in-tree product
LIB_PATH = os.environ.get("QI_LIB_PATH") or os.path.join(HERE,
                                                         "libquadiron_amd.so")

_lib = None

c_u8p = C.POINTER(C.c_uint8)
c_u8pp = C.POINTER(c_u8p)


def _declare(lib):
    V, I, LL, SZ, U32 = C.c_void_p, C.c_int, C.c_longlong, C.c_size_t, C.c_uint32
    sig = {
        # include/quadiron_c.h
        "quadiron_fnt32_new": (V, [I, I, I, I]),
        "quadiron_fnt32_delete": (None, [V]),
        "quadiron_fnt32_get_metadata_size": (I, [V, SZ]),
        "quadiron_fnt32_encode": (I, [V, c_u8pp, c_u8pp, V, SZ]),
        "quadiron_fnt32_decode": (I, [V, c_u8pp, c_u8pp, V, SZ]),
        "quadiron_fnt32_reconstruct": (I, [V, c_u8pp, c_u8pp, V, C.c_uint, SZ]),
        "quadiron_hex_dump": (None, [V, SZ]),
        # include/qi_gpu.h
        "qi_gpu_device_count": (I, []),
        "qi_plan_create": (V, [I, I, I]),
        "qi_plan_create_ex": (V, [I, I, I, I]),
        "qi_plan_destroy": (None, [V]),
        "qi_plan_n": (I, [V]),
        "qi_plan_n_outputs": (I, [V]),
        "qi_gpu_oor_clear": (I, [V, SZ, V]),
        "qi_gpu_encode": (I, [V, V, LL, LL, V, LL, LL, LL, I, V, V, I, V]),
        "qi_gpu_decode_ctx_bytes": (SZ, [V, I, LL]),
        "qi_gpu_decode_ctx": (I, [V, V, V, I, V, V, I, LL, V, V]),
        "qi_gpu_decode": (I, [V, V, V, V, LL, LL, V, LL, LL, V, V, I, V, LL,
                              LL, LL, I, V]),
        "qi_gpu_decode_ctx_packed": (I, [V, V, V, I, V, V, I, LL, V, V]),
        "qi_gpu_decode_packed": (I, [V, V, V, LL, LL, V, V, I, V, LL, LL, LL,
                                     I, V]),
        "qi_gpu_take_error": (I, [V]),
        "qi_build_id": (C.c_char_p, []),
        "qi_gpu_kernels": (C.c_char_p, [V, LL]),
        "qi_fec_new": (V, [I, I, I]),
        "qi_fec_delete": (None, [V]),
        "qi_fec_n_outputs": (I, [V]),
        "qi_fec_encode_blocks": (I, [V, c_u8pp, c_u8pp, SZ, V, V, U32]),
        "qi_fec_decode_blocks": (I, [V, c_u8pp, c_u8pp, V, V, U32, V, V, SZ]),
        "qi_fec_encode_streams": (I, [V, c_u8pp, SZ, c_u8pp, V, V, U32]),
        "qi_fec_decode_streams": (I, [V, c_u8pp, c_u8pp, SZ, V, V, U32,
                                      c_u8pp]),
        "qi_nf4_new": (V, [I, I, I]),
        "qi_nf4_delete": (None, [V]),
        "qi_nf4_n_outputs": (I, [V]),
        "qi_nf4_encode_blocks": (I, [V, c_u8pp, c_u8pp, SZ, V, V, V, U32]),
        "qi_nf4_decode_blocks": (I, [V, c_u8pp, c_u8pp, V, V, V, U32, V, V,
                                     SZ]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def lib():
    """Load the native library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} missing: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` or "
                "`make -C quadiron_amd/csrc`")
        # torch-rocm bundles its own libamdhip64 with the same SONAME
        # (libamdhip64.so.7): load torch first so the process keeps ONE HIP
        # runtime (ours then binds to it) and torch streams/pointers are
        # valid in our launches.  C-ABI users without torch get /opt/rocm's.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _lib = _declare(C.CDLL(LIB_PATH))
    return _lib


def build_id():
    """'<git describe>+src:<source hash>' baked into the loaded library."""
    return lib().qi_build_id().decode()


def _rows(t, name, rows=None, stripes=None):
    """Check a [S, rows, P] u16 row tensor before its pointer and strides go
    to the device C-ABI: a wrong dtype, device, shape or a non-unit inner
    stride would become out-of-bounds device accesses."""
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name}: expected a HIP (cuda) tensor")
    if t.dtype not in (torch.int16, torch.uint16):
        raise TypeError(f"{name}: expected int16/uint16, got {t.dtype}")
    if t.dim() != 3 or t.stride(-1) != 1:
        raise ValueError(f"{name}: expected [S, rows, P] with unit inner stride")
    if rows is not None and t.shape[1] != rows:
        raise ValueError(f"{name}: expected {rows} rows, got {t.shape[1]}")
    if stripes is not None and t.shape[0] != stripes:
        raise ValueError(f"{name}: expected {stripes} stripes, got {t.shape[0]}")


def _flat(t, name, n, dtypes):
    """A device buffer of at least n elements of one of `dtypes`."""
    if t is None:
        return
    if not t.is_cuda or t.dtype not in dtypes or not t.is_contiguous():
        raise TypeError(f"{name}: expected a contiguous HIP tensor of {dtypes}")
    if t.numel() < n:
        raise ValueError(f"{name}: {t.numel()} elements, need {n}")


def _oor(counts, entries, cap, S, slots):
    import torch
    if counts is None:
        return
    if entries is None or cap < 1:
        raise ValueError("OOR buckets need counts, entries and cap >= 1")
    _flat(counts, "counts", S * slots, (torch.int32,))
    _flat(entries, "entries", S * slots * cap, (torch.int32,))


def require_device():
    n = lib().qi_gpu_device_count()
    if n < 1:
        raise RuntimeError("quadiron_amd: no HIP device visible")
    return n


def ptr_array(arrs):
    """uint8_t** from a list of numpy uint8 arrays (None -> NULL)."""
    p = (c_u8p * len(arrs))()
    for i, a in enumerate(arrs):
        p[i] = a.ctypes.data_as(c_u8p) if a is not None else None
    return p


class Plan:
    """Device plan (include/qi_gpu.h) for RS-FNT(k, m)."""

    ENCODERS = {None: 0, "matrix": 1, "codelets": 2}  # QI_PLAN_ENC_* flags

    def __init__(self, k, m, systematic=False, encoder=None):
        """encoder: None (the library's choice), "matrix" or "codelets"
        (force the non-systematic encode kernel for k <= 64)."""
        require_device()
        if encoder not in self.ENCODERS:
            raise ValueError(f"encoder must be one of {list(self.ENCODERS)}")
        self.k, self.m, self.sys = k, m, bool(systematic)
        self.h = lib().qi_plan_create_ex(k, m, int(systematic),
                                         self.ENCODERS[encoder])
        if not self.h:
            raise ValueError(f"qi_plan_create({k}, {m}, {systematic}) failed")
        self.n = lib().qi_plan_n(self.h)
        self.n_outputs = lib().qi_plan_n_outputs(self.h)

    def kernels(self, words):
        """'encode=<kernels>; decode=<kernels>' this plan launches over
        `words` columns (qi_gpu_kernels)."""
        return lib().qi_gpu_kernels(self.h, words).decode()

    def close(self):
        if self.h:
            lib().qi_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _stream(stream):
        return stream if stream is not None else None

    def encode(self, data, out, counts=None, entries=None, cap=0, stream=None):
        """data: int16/uint16 tensor [S, k, P] on cuda; out: [S, n_out, P]."""
        _rows(data, "data", self.k)
        S, k, P = data.shape
        _rows(out, "out", self.n_outputs, S)
        if out.shape[2] < P:
            raise ValueError("out: fewer columns than data")
        _oor(counts, entries, cap, S, self.n_outputs)
        rc = lib().qi_gpu_encode(
            self.h, data.data_ptr(), data.stride(0), data.stride(1),
            out.data_ptr(), out.stride(0), out.stride(1), P, S,
            counts.data_ptr() if counts is not None else None,
            entries.data_ptr() if entries is not None else None, int(cap),
            self._stream(stream))
        if rc:
            raise RuntimeError(f"qi_gpu_encode failed: {rc}")

    def ctx_bytes(self, n_stripes, words):
        return lib().qi_gpu_decode_ctx_bytes(self.h, n_stripes, words)

    def decode_ctx(self, ids, ctx, words, counts=None, entries=None, cap=0,
                   h_ids=None, stream=None):
        """ids: int16 tensor [S, k] on cuda (fragment ids); OOR buckets of
        the coded rows as produced by encode (routed into the contexts)."""
        import torch
        S = ids.shape[0]
        _flat(ids, "ids", S * self.k, (torch.int16, torch.uint16))
        _flat(ctx, "ctx", self.ctx_bytes(S, words), (torch.uint8,))
        _oor(counts, entries, cap, S, self.n_outputs)
        rc = lib().qi_gpu_decode_ctx(
            self.h, ids.data_ptr(),
            h_ids.ctypes.data_as(C.c_void_p) if h_ids is not None else None,
            ids.shape[0],
            counts.data_ptr() if counts is not None else None,
            entries.data_ptr() if entries is not None else None, int(cap),
            words, ctx.data_ptr(), self._stream(stream))
        if rc:
            raise RuntimeError(f"qi_gpu_decode_ctx failed: {rc}")

    def decode(self, ctx, ids, coded, out, data=None, counts=None,
               entries=None, cap=0, stream=None, check=True):
        """coded: [S, n_out, P] (fragment slot rows); out: [S, k, P].
        check: synchronise and return the sticky OOR-overflow flag
        (qi_gpu_take_error); with check=False the call stays asynchronous
        and returns 0 -- call take_error() later."""
        import torch
        _rows(out, "out", self.k)
        S, _, P = out.shape
        _rows(coded, "coded", self.n_outputs, S)
        if data is not None:
            _rows(data, "data", self.k, S)
        _flat(ids, "ids", S * self.k, (torch.int16, torch.uint16))
        _flat(ctx, "ctx", self.ctx_bytes(S, P), (torch.uint8,))
        _oor(counts, entries, cap, S, self.n_outputs)
        d = data if data is not None else coded
        rc = lib().qi_gpu_decode(
            self.h, ctx.data_ptr(), ids.data_ptr(), d.data_ptr(), d.stride(0),
            d.stride(1), coded.data_ptr(), coded.stride(0), coded.stride(1),
            counts.data_ptr() if counts is not None else None,
            entries.data_ptr() if entries is not None else None, int(cap),
            out.data_ptr(), out.stride(0), out.stride(1), P, S,
            self._stream(stream))
        if rc:
            raise RuntimeError(f"qi_gpu_decode failed: {rc}")
        return lib().qi_gpu_take_error(self.h) if check else 0

    def decode_ctx_packed(self, ids, ctx, words, counts=None, entries=None,
                          cap=0, h_ids=None, stream=None):
        """Contexts for decode_packed: OOR buckets indexed by the position
        of the received row (slots = k)."""
        import torch
        S = ids.shape[0]
        _flat(ids, "ids", S * self.k, (torch.int16, torch.uint16))
        _flat(ctx, "ctx", self.ctx_bytes(S, words), (torch.uint8,))
        _oor(counts, entries, cap, S, self.k)
        rc = lib().qi_gpu_decode_ctx_packed(
            self.h, ids.data_ptr(),
            h_ids.ctypes.data_as(C.c_void_p) if h_ids is not None else None,
            ids.shape[0],
            counts.data_ptr() if counts is not None else None,
            entries.data_ptr() if entries is not None else None, int(cap),
            words, ctx.data_ptr(), self._stream(stream))
        if rc:
            raise RuntimeError(f"qi_gpu_decode_ctx_packed failed: {rc}")

    def decode_packed(self, ctx, recv, out, counts=None, entries=None, cap=0,
                      stream=None, check=True):
        """recv: [S, k, P] received rows in id order; out: [S, k, P]."""
        import torch
        _rows(out, "out", self.k)
        S, _, P = out.shape
        _rows(recv, "recv", self.k, S)
        _flat(ctx, "ctx", self.ctx_bytes(S, P), (torch.uint8,))
        _oor(counts, entries, cap, S, self.k)
        rc = lib().qi_gpu_decode_packed(
            self.h, ctx.data_ptr(), recv.data_ptr(), recv.stride(0),
            recv.stride(1),
            counts.data_ptr() if counts is not None else None,
            entries.data_ptr() if entries is not None else None, int(cap),
            out.data_ptr(), out.stride(0), out.stride(1), P, S,
            self._stream(stream))
        if rc:
            raise RuntimeError(f"qi_gpu_decode_packed failed: {rc}")
        return lib().qi_gpu_take_error(self.h) if check else 0

    def take_error(self):
        return lib().qi_gpu_take_error(self.h)


class Fec:
    """Block API (qi::fec::RsFnt via the qi_fec_* C view)."""

    def __init__(self, k, m, systematic=False):
        require_device()
        self.k, self.m, self.sys = k, m, bool(systematic)
        self.h = lib().qi_fec_new(int(systematic), k, m)
        if not self.h:
            raise ValueError("qi_fec_new failed")
        self.n_outputs = lib().qi_fec_n_outputs(self.h)

    def close(self):
        if self.h:
            lib().qi_fec_delete(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Nf4:
    """RS-NF4 block API (qi::fec::RsNf4 via the qi_nf4_* C view)."""

    def __init__(self, word_size, k, m):
        require_device()
        self.ws, self.k, self.m = word_size, k, m
        self.h = lib().qi_nf4_new(word_size, k, m)
        if not self.h:
            raise ValueError(f"qi_nf4_new({word_size}, {k}, {m}) failed")
        self.n_outputs = lib().qi_nf4_n_outputs(self.h)

    def encode(self, data, outputs, oor, flags, counts):
        """data: k uint8 rows; outputs: n_outputs rows (None = unwanted);
        oor/flags: (n_outputs, cap) uint32; counts: (n_outputs,) uint32."""
        rc = lib().qi_nf4_encode_blocks(
            self.h, ptr_array(data), ptr_array(outputs), len(data[0]),
            oor.ctypes.data_as(C.c_void_p), flags.ctypes.data_as(C.c_void_p),
            counts.ctypes.data_as(C.c_void_p), oor.shape[1])
        if rc:
            raise RuntimeError(f"qi_nf4_encode_blocks failed: {rc}")

    def decode(self, data, parities, oor, flags, counts, missing, wanted):
        """Returns 1 (decoded) or 0 (fewer than k fragments)."""
        rc = lib().qi_nf4_decode_blocks(
            self.h, ptr_array(data), ptr_array(parities),
            oor.ctypes.data_as(C.c_void_p), flags.ctypes.data_as(C.c_void_p),
            counts.ctypes.data_as(C.c_void_p), oor.shape[1],
            missing.ctypes.data_as(C.c_void_p),
            wanted.ctypes.data_as(C.c_void_p), len(data[0]))
        if rc < 0:
            raise RuntimeError(f"qi_nf4_decode_blocks failed: {rc}")
        return rc

    def close(self):
        if self.h:
            lib().qi_nf4_delete(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class QuadironFnt32:
    """The drop-in C-ABI handle (include/quadiron_c.h)."""

    def __init__(self, word_size, n_data, n_parities, systematic):
        self.h = lib().quadiron_fnt32_new(word_size, n_data, n_parities,
                                          int(systematic))
        if not self.h:
            raise ValueError("quadiron_fnt32_new returned NULL")
        self.k, self.m, self.sys = n_data, n_parities, bool(systematic)

    def metadata_size(self, block_size):
        return lib().quadiron_fnt32_get_metadata_size(self.h, block_size)

    def encode(self, data, parity, wanted, block_size):
        return lib().quadiron_fnt32_encode(
            self.h, ptr_array(data), ptr_array(parity),
            wanted.ctypes.data_as(C.c_void_p), block_size)

    def decode(self, data, parity, missing, block_size):
        return lib().quadiron_fnt32_decode(
            self.h, ptr_array(data), ptr_array(parity),
            missing.ctypes.data_as(C.c_void_p), block_size)

    def reconstruct(self, data, parity, missing, dest, block_size):
        return lib().quadiron_fnt32_reconstruct(
            self.h, ptr_array(data), ptr_array(parity),
            missing.ctypes.data_as(C.c_void_p), dest, block_size)

    def close(self):
        if self.h:
            lib().quadiron_fnt32_delete(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
