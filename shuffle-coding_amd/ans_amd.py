"""Python binding of libshufflecoding_amd.so (include/ans_capi.h) via ctypes.

Mirrors the reference's coder surface with the same names and argument meaning:
  Message.zeros/empty/random/unflatten, flatten, bits, virtual_bits, ==   src/ans.rs:225-310
  Codec.push/pop/bits/sample/samples, test_invertibility/test             src/ans.rs:28-75
  Distribution (norm/pmf/cdf/icdf) through the two-phase scalar ABI       src/ans.rs:80-121
  Uniform / Categorical / Bernoulli / IID / Independent                   src/codec.rs
and exposes the GPU bulk path (section 4 of the header): GpuTable.encode_chunks /
decode_chunks on host buffers and dev_encode / dev_decode / dev_gen_iid on device
memory (torch tensors or raw pointers).

There is no CPU fallback for the GPU path: if the shared library or the GPU is missing,
the calls raise.
"""
import collections
import ctypes
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SHUFFLE_CODING_AMD_LIB selects another build of the same library (A/B experiments)
LIB_PATH = os.environ.get("SHUFFLE_CODING_AMD_LIB") or os.path.join(HERE, "lib", "libshufflecoding_amd.so")

ANS_OK, ANS_E_ZERO_MASS, ANS_E_EXHAUSTED, ANS_E_LEN, ANS_E_SYMBOL = 0, 1, 2, 3, 4
ANS_E_NORM_RANGE, ANS_E_DEVICE, ANS_E_ALLOC, ANS_E_ARG, ANS_E_MISMATCH = 5, 6, 7, 8, 9
GEN_ZEROS, GEN_EMPTY, GEN_RANDOM = 0, 1, 2
ANS_PATH_ENC_LDS, ANS_PATH_ENC_GLOBAL, ANS_PATH_DEC_LDS, ANS_PATH_DEC_GLOBAL = 1, 2, 4, 8
ANS_PATH_ENC_WIDE, ANS_PATH_DEC_WIDE = 16, 32
ANS_PATH_DEC_COMPACT = 64
ANS_PATH_ENC_PACKED = 128
ANS_PATH_DEC_U = 256
ANS_PATH_ENC_SHIFT = 512
MAX_MIN_HEAD = 1 << 56
MAX_SIZE = MAX_MIN_HEAD >> 10

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p
u64 = ctypes.c_uint64
sz = ctypes.c_size_t
ci = ctypes.c_int

# name -> (restype, argtypes); this list is also the ABI-export test's expectation.
SIGNATURES = {
    "ans_status_string": (ctypes.c_char_p, [ci]),
    "ans_abi_version": (ci, []),
    "ans_msg_new": (ci, [ci, u64, ctypes.POINTER(vp)]),
    "ans_msg_free": (None, [vp]),
    "ans_msg_clone": (ci, [vp, ctypes.POINTER(vp)]),
    "ans_msg_flatten": (ci, [vp, vp, sz, ctypes.POINTER(sz)]),
    "ans_msg_unflatten": (ci, [vp, sz, ci, u64, ctypes.POINTER(vp)]),
    "ans_msg_reflatten": (ci, [vp, ctypes.POINTER(vp)]),
    "ans_msg_bits": (ci, [vp, u64p]),
    "ans_msg_virtual_bits": (ci, [vp, ctypes.POINTER(ctypes.c_double)]),
    "ans_msg_equal": (ci, [vp, vp, ctypes.POINTER(ci)]),
    "ans_msg_state": (ci, [vp, u64p, u64p, u64p]),
    "ans_push_begin": (ci, [vp, u64, u64, u64p, u64p]),
    "ans_push_end": (ci, [vp, u64, u64, u64]),
    "ans_pop_begin": (ci, [vp, u64, u64p, u64p]),
    "ans_pop_end": (ci, [vp, u64, u64, u64]),
    "ans_uniform_push": (ci, [vp, u64, u64]),
    "ans_uniform_pop": (ci, [vp, u64, u64p]),
    "ans_table_create": (ci, [vp, ctypes.c_uint32, ctypes.POINTER(vp)]),
    "ans_table_create_bernoulli": (ci, [u64, u64, ctypes.POINTER(vp)]),
    "ans_table_free": (None, [vp]),
    "ans_table_info": (ci, [vp, u32p, u64p]),
    "ans_cat_push": (ci, [vp, vp, u64]),
    "ans_cat_pop": (ci, [vp, vp, u64p]),
    "ans_push_iid": (ci, [vp, vp, vp, sz]),
    "ans_pop_iid": (ci, [vp, vp, vp, sz]),
    "ans_gpu_device_count": (ci, [ctypes.POINTER(ci)]),
    "ans_gpu_create": (ci, [ci, ctypes.POINTER(vp)]),
    "ans_gpu_free": (None, [vp]),
    "ans_gpu_set_batch_bytes": (ci, [vp, u64]),
    "ans_gpu_pipe_depth": (ci, [vp, ctypes.POINTER(ci)]),
    "ans_host_alloc": (ci, [sz, ctypes.POINTER(vp)]),
    "ans_host_free": (None, [vp]),
    "ans_gpu_table_create": (ci, [vp, vp, ctypes.POINTER(vp)]),
    "ans_gpu_table_free": (None, [vp]),
    "ans_gpu_slot_capacity": (ci, [vp, u64, u64p]),
    "ans_gpu_table_paths": (ci, [vp, ctypes.POINTER(ctypes.c_uint32)]),
    "ans_gpu_encode_chunks_ex": (ci, [vp, vp, ci, u64, u64, ci, u64, vp, u64, vp, vp, u64p]),
    "ans_gpu_decode_chunks_ex": (ci, [vp, vp, u64, vp, vp, u64, u64, ci, u64, vp, ci]),
    "ans_dev_encode_chunks_ex": (ci, [vp, vp, ci, u64, u64, ci, u64, vp, u64, vp, vp, vp]),
    "ans_dev_decode_chunks_ex": (ci, [vp, vp, vp, u64, vp, u64, u64, ci, u64, vp, ci, vp, vp]),
    "ans_gpu_encode_var_chunks_ex": (ci, [vp, vp, ci, u64, vp, ci, u64, vp, u64, vp, vp, u64p]),
    "ans_gpu_decode_var_chunks_ex": (ci, [vp, vp, u64, vp, vp, u64, vp, ci, u64, vp, ci]),
    "ans_dev_encode_var_chunks_ex": (ci, [vp, vp, ci, u64, vp, ci, u64, vp, u64, vp, vp, vp]),
    "ans_dev_decode_var_chunks_ex": (ci, [vp, vp, vp, u64, vp, u64, vp, ci, u64, vp, ci, vp, vp]),
    "ans_gpu_uniform_encode_chunks": (ci, [vp, u64, vp, ci, u64, u64, ci, u64, vp, u64, vp, vp, u64p]),
    "ans_gpu_uniform_decode_chunks": (ci, [vp, u64, vp, u64, vp, vp, u64, u64, ci, u64, vp, ci]),
    "ans_gpu_loguniform_encode_chunks": (ci, [vp, ctypes.c_uint32, vp, ci, u64, u64, ci, u64, vp, u64, vp, vp, u64p]),
    "ans_gpu_loguniform_decode_chunks": (ci, [vp, ctypes.c_uint32, vp, u64, vp, vp, u64, u64, ci, u64, vp, ci]),
    "ans_gpu_tableset_create": (ci, [vp, ctypes.POINTER(vp), ctypes.c_uint32, ctypes.POINTER(vp)]),
    "ans_gpu_tableset_free": (None, [vp]),
    "ans_gpu_independent_encode_chunks": (ci, [vp, vp, vp, ci, u64, u64, ci, u64, vp, u64, vp, vp, u64p]),
    "ans_gpu_independent_decode_chunks": (ci, [vp, vp, vp, u64, vp, vp, u64, u64, ci, u64, vp, ci]),
    "ans_gpu_tableset_fast": (ci, [vp, ctypes.POINTER(ci)]),
    "ans_gpu_tableset_lanes": (ci, [vp, ci]),
    "ans_gpu_uniform_slot_capacity": (ci, [u64, u64, ctypes.POINTER(u64)]),
    "ans_gpu_loguniform_slot_capacity": (ci, [ctypes.c_uint32, u64, ctypes.POINTER(u64)]),
    "ans_gpu_tableset_slot_capacity": (ci, [vp, u64, ctypes.POINTER(u64)]),
    "ans_dev_uniform_encode": (ci, [vp, u64, vp, ci, u64, u64, ci, u64, vp, u64, vp, vp, vp]),
    "ans_dev_uniform_decode": (ci, [vp, u64, vp, vp, u64, vp, u64, u64, ci, u64, vp, ci, vp, vp]),
    "ans_dev_loguniform_encode": (ci, [vp, ctypes.c_uint32, vp, ci, u64, u64, ci, u64, vp, u64, vp, vp, vp]),
    "ans_dev_loguniform_decode": (ci, [vp, ctypes.c_uint32, vp, vp, u64, vp, u64, u64, ci, u64, vp, ci, vp, vp]),
    "ans_dev_independent_encode": (ci, [vp, vp, vp, ci, u64, u64, ci, u64, vp, u64, vp, vp, vp]),
    "ans_dev_independent_decode": (ci, [vp, vp, vp, vp, u64, vp, u64, u64, ci, u64, vp, ci, vp, vp]),
    "ans_gpu_encode_chunks": (ci, [vp, vp, ci, u64, u64, vp, u64, vp, vp, u64p]),
    "ans_gpu_decode_chunks": (ci, [vp, vp, u64, vp, vp, u64, u64, ci, vp, ci]),
    "ans_dev_encode_chunks": (ci, [vp, vp, ci, u64, u64, vp, u64, vp, vp, vp]),
    "ans_dev_decode_chunks": (ci, [vp, vp, vp, u64, vp, u64, u64, ci, vp, ci, vp, vp]),
    "ans_dev_gen_iid": (ci, [vp, u64, u64, u64, vp, ci, vp]),
    "ans_dev_compact": (ci, [vp, vp, u64, vp, vp, u64, vp, vp]),
    "ans_dense_offsets_entries": (u64, [u64]),
    "ans_dev_encode_dense": (ci, [vp, vp, ci, u64, u64, vp, u64, vp, vp, vp, u64, vp, vp]),
    "ans_dev_encode_dense_ex": (ci, [vp, vp, ci, u64, u64, ci, u64, vp, u64, vp, vp, vp, u64, vp, vp]),
    "ans_dev_status": (ci, [vp, vp, vp, ctypes.POINTER(ci)]),
    "ans_dev_expand": (ci, [vp, vp, vp, vp, u64, vp, u64, vp]),
    "ans_dev_sample_iid": (ci, [vp, u64, u64, u64, vp, ci, vp]),
    "ans_dev_check_renorm": (ci, [vp, vp, vp, u64, u64, vp, vp, vp]),
    "ans_gpu_sample_iid": (ci, [vp, u64, u64, u64, vp, ci]),
    "ans_edge_alphabet_len": (ci, [u64, ci, ci, u64p]),
    "ans_dev_edges_to_dense": (ci, [vp, u64, ci, ci, vp, u64, vp, vp, vp]),
    "ans_dev_dense_to_edges": (ci, [vp, u64, ci, ci, vp, vp, u64, vp, vp, vp]),
    "ans_gpu_dense_set_encode": (ci, [vp, u64, ci, ci, vp, u64, u64, vp, u64, vp, vp, u64p]),
    "ans_gpu_dense_set_decode": (ci, [vp, u64, ci, ci, vp, u64, vp, vp, u64, vp, u64, u64p]),
    "ans_dev_encode_var_chunks": (ci, [vp, vp, ci, u64, vp, vp, u64, vp, vp, vp]),
    "ans_dev_decode_var_chunks": (ci, [vp, vp, vp, u64, vp, u64, vp, ci, vp, ci, vp, vp]),
    "ans_gpu_encode_var_chunks": (ci, [vp, vp, ci, u64, vp, vp, u64, vp, vp, u64p]),
    "ans_gpu_decode_var_chunks": (ci, [vp, vp, u64, vp, vp, u64, vp, ci, vp, ci]),
    "ans_gpu_dense_sets_encode": (ci, [vp, u64, vp, ci, ci, vp, vp, vp, u64, vp, vp, u64p]),
    "ans_gpu_dense_sets_decode": (ci, [vp, u64, vp, ci, ci, vp, u64, vp, vp, vp, u64, vp]),
    "ans_gpu_independent_encode_var_chunks": (ci, [vp, vp, vp, ci, u64, vp, ci, u64, vp, u64, vp, vp, u64p]),
    "ans_gpu_independent_decode_var_chunks": (ci, [vp, vp, vp, u64, vp, vp, u64, vp, ci, u64, vp, ci]),
    "ans_dev_independent_encode_var": (ci, [vp, vp, vp, ci, u64, vp, ci, u64, vp, u64, vp, vp, vp]),
    "ans_dev_independent_decode_var": (ci, [vp, vp, vp, vp, u64, vp, u64, vp, ci, u64, vp, ci, vp, vp]),
    "ans_gpu_graphs_encode": (ci, [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ci, ci, u64, vp, vp, vp, vp,
                                   vp, ci, u64, vp, u64, vp, vp, u64p]),
    "ans_gpu_graphs_decode": (ci, [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ci, ci, u64, vp, vp, u64, vp,
                                   vp, ci, u64, vp, vp, vp, u64, vp]),
}
ANS_NO_TABLE = 0xFFFFFFFF

_lib = None


class AnsError(RuntimeError):
    def __init__(self, code, where=""):
        self.code = code
        msg = lib().ans_status_string(code).decode() if _lib is not None else str(code)
        super().__init__(f"{where}: {msg} (status {code})" if where else f"{msg} (status {code})")


def lib():
    """Loads the in-tree shared library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `make -C shuffle-coding_amd` (or __graft_entry__.build())")
        # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same soname).
        # Loading torch first makes the dynamic loader bind our library to that copy, so
        # device pointers and streams from torch are valid in our kernels.  Without torch
        # the library binds to /opt/rocm's runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(rc, where=""):
    if rc != ANS_OK:
        raise AnsError(rc, where)


def _np_ptr(a):
    return a.ctypes.data_as(vp)


# ============================================================== Message (src/ans.rs:225-310)
class Message:
    __slots__ = ("h",)

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def _new(cls, kind, seed=0):
        h = vp()
        _check(lib().ans_msg_new(kind, seed, ctypes.byref(h)), "Message::new")
        return cls(h)

    @classmethod
    def zeros(cls):
        return cls._new(GEN_ZEROS)

    @classmethod
    def empty(cls):
        return cls._new(GEN_EMPTY)

    @classmethod
    def random(cls, seed):
        return cls._new(GEN_RANDOM, seed)

    @classmethod
    def unflatten(cls, data, kind=GEN_ZEROS, seed=0):
        buf = np.frombuffer(bytes(data), dtype=np.uint8)
        h = vp()
        _check(lib().ans_msg_unflatten(_np_ptr(buf) if len(buf) else None, len(buf), kind, seed, ctypes.byref(h)),
               "Message::unflatten")
        return cls(h)

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:
            _lib.ans_msg_free(h)
            self.h = None

    def clone(self):
        h = vp()
        _check(lib().ans_msg_clone(self.h, ctypes.byref(h)), "Message::clone")
        return Message(h)

    def flatten(self):
        n = sz(0)
        _check(lib().ans_msg_flatten(self.h, None, 0, ctypes.byref(n)), "Message::flatten")
        buf = np.zeros(max(n.value, 1), np.uint8)
        _check(lib().ans_msg_flatten(self.h, _np_ptr(buf), n.value, ctypes.byref(n)), "Message::flatten")
        return bytes(buf[:n.value])

    def reflatten(self):
        """Message::unflatten(self.clone().flatten()) with the tail's generator kept (src/ans.rs:57)."""
        h = vp()
        _check(lib().ans_msg_reflatten(self.h, ctypes.byref(h)), "Message::unflatten(flatten)")
        return Message(h)

    def bits(self):
        b = u64(0)
        _check(lib().ans_msg_bits(self.h, ctypes.byref(b)), "Message::bits")
        return b.value

    def virtual_bits(self):
        b = ctypes.c_double(0)
        _check(lib().ans_msg_virtual_bits(self.h, ctypes.byref(b)), "Message::virtual_bits")
        return b.value

    def state(self):
        h, t, g = u64(0), u64(0), u64(0)
        _check(lib().ans_msg_state(self.h, ctypes.byref(h), ctypes.byref(t), ctypes.byref(g)))
        return h.value, t.value, g.value

    @property
    def head(self):
        return self.state()[0]

    def __eq__(self, other):
        e = ci(0)
        _check(lib().ans_msg_equal(self.h, other.h, ctypes.byref(e)), "Message::eq")
        return bool(e.value)

    def __ne__(self, other):
        return not self == other


# ============================================================== Codec trait (src/ans.rs:28-75)
CodecTestResults = collections.namedtuple("CodecTestResults", "bits amortized_bits enc_sec dec_sec")


def assert_bits_close(expected_bits, bits, tol):  # src/ans.rs:329-332
    mismatch = abs(bits - expected_bits) / max(abs(expected_bits), 1.0)
    assert mismatch < tol, f"Expected {expected_bits} bits, but got {bits} bits."


def assert_bits_eq(expected_bits, bits):  # src/ans.rs:325-327
    assert_bits_close(expected_bits, bits, 1e-5)


class Codec:
    def push(self, m, x):
        raise NotImplementedError

    def pop(self, m):
        raise NotImplementedError

    def bits(self, x):
        return None

    def sample(self, seed):  # src/ans.rs:38-40
        return self.pop(Message.random(seed))

    def samples(self, length, seed):  # src/ans.rs:42-44
        return IID(self, length).sample(seed)

    def test_invertibility(self, x, initial):  # src/ans.rs:47-59
        import time
        m = initial.clone()
        t0 = time.perf_counter()
        self.push(m, x)
        enc_sec = time.perf_counter() - t0
        bits = m.bits()
        amortized_bits = m.virtual_bits() - initial.virtual_bits()
        assert bits >= amortized_bits
        t0 = time.perf_counter()
        decoded = self.pop(m)
        dec_sec = time.perf_counter() - t0
        assert _sym_eq(x, decoded), "decoded != x"
        assert initial == m, "message did not return to its initial state"
        assert initial == m.reflatten(), "flatten/unflatten round trip"
        return CodecTestResults(bits, amortized_bits, enc_sec, dec_sec)

    def test(self, x, initial):  # src/ans.rs:62-68
        out = self.test_invertibility(x, initial)
        b = self.bits(x)
        if b is not None:
            assert_bits_eq(b, out.amortized_bits)
        return out

    def test_on_samples(self, num_samples):  # src/ans.rs:72-74
        return [self.test(self.sample(seed), Message.random(seed)).amortized_bits for seed in range(num_samples)]


def _sym_eq(a, b):
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return np.array_equal(np.asarray(a), np.asarray(b))
    return a == b


class Distribution(Codec):
    """A Python Distribution (norm/pmf/cdf/icdf) coded through the two-phase scalar ABI,
    exactly as the blanket `impl<D: Distribution> Codec for D` (src/ans.rs:93-121)."""

    def norm(self):
        raise NotImplementedError

    def pmf(self, x):
        raise NotImplementedError

    def cdf(self, x, i):
        raise NotImplementedError

    def icdf(self, cf):
        raise NotImplementedError

    def push(self, m, x):
        q, r = u64(0), u64(0)
        _check(lib().ans_push_begin(m.h, self.pmf(x), self.norm(), ctypes.byref(q), ctypes.byref(r)), "push")
        _check(lib().ans_push_end(m.h, self.norm(), q.value, self.cdf(x, r.value)), "push")

    def pop(self, m):
        q, cf = u64(0), u64(0)
        _check(lib().ans_pop_begin(m.h, self.norm(), ctypes.byref(q), ctypes.byref(cf)), "pop")
        x, r = self.icdf(cf.value)
        _check(lib().ans_pop_end(m.h, self.pmf(x), q.value, r), "pop")
        return x

    def bits(self, x):  # src/ans.rs:118-120
        return math.log2(self.norm()) - math.log2(self.pmf(x))


class Uniform(Distribution):  # src/codec.rs:13-49
    def __init__(self, size):
        assert size <= MAX_SIZE
        self.size = size

    def norm(self):
        return self.size

    def pmf(self, x):
        return 1

    def cdf(self, x, i):
        assert i == 0
        return x

    def icdf(self, cf):
        return cf, 0

    def push(self, m, x):
        _check(lib().ans_uniform_push(m.h, self.size, x), "Uniform::push")

    def pop(self, m):
        x = u64(0)
        _check(lib().ans_uniform_pop(m.h, self.size, ctypes.byref(x)), "Uniform::pop")
        return x.value

    def uni_bits(self):
        return math.log2(self.size)


class LogUniform(Codec):  # src/codec.rs:561-611 (MaxBenfordIID's item, src/param_codec.rs:117-119)
    """x's bit length is Uniform over [0, excl_max_bits]; the bits below the top one are
    Uniform(2^(bits-1)), pushed first."""

    def __init__(self, excl_max_bits):
        assert excl_max_bits <= 64
        self.bits_codec = Uniform(excl_max_bits + 1)

    @classmethod
    def max(cls):  # LogUniform::new(47)
        return cls(47)

    @staticmethod
    def get_bits(x):
        return int(x).bit_length()

    def push(self, m, x):
        b = self.get_bits(x)
        assert b < self.bits_codec.size
        if b:
            size = 1 << (b - 1)
            Uniform(size).push(m, int(x) & ~size)
        self.bits_codec.push(m, b)

    def pop(self, m):
        b = self.bits_codec.pop(m)
        if b == 0:
            return 0
        size = 1 << (b - 1)
        return Uniform(size).pop(m) | size

    def bits(self, x):
        b = self.get_bits(x)
        return self.bits_codec.uni_bits() + (Uniform(1 << (b - 1)).uni_bits() if b else 0.0)


class Categorical(Distribution):  # src/codec.rs:51-92
    def __init__(self, masses):
        self.masses = np.ascontiguousarray(np.asarray(masses, dtype=np.uint64))
        self.cummasses = np.concatenate([[0], np.cumsum(self.masses)[:-1]]).astype(np.uint64) if len(
            self.masses) else np.zeros(0, np.uint64)
        self._norm = int(self.masses.sum()) if len(self.masses) else 0
        h = vp()
        _check(lib().ans_table_create(_np_ptr(self.masses), len(self.masses), ctypes.byref(h)), "Categorical::new")
        self.table = h

    def __del__(self):
        h = getattr(self, "table", None)
        if h and _lib is not None:
            _lib.ans_table_free(h)
            self.table = None

    def norm(self):
        return self._norm

    def pmf(self, x):
        return int(self.masses[x])

    def cdf(self, x, i):
        return int(self.cummasses[x]) + i

    def icdf(self, cf):
        x = int(np.searchsorted(self.cummasses, cf, side="right")) - 1
        return x, cf - int(self.cummasses[x])

    def push(self, m, x):
        _check(lib().ans_cat_push(m.h, self.table, int(x)), "Categorical::push")

    def pop(self, m):
        x = u64(0)
        _check(lib().ans_cat_pop(m.h, self.table, ctypes.byref(x)), "Categorical::pop")
        return x.value

    def prob(self, x):
        return int(self.masses[x]) / self._norm

    def entropy(self):
        p = self.masses.astype(np.float64) / self._norm
        p = p[p > 0]
        return float(-(p * np.log2(p)).sum())


class Bernoulli(Distribution):  # src/codec.rs:94-129
    def __init__(self, mass, norm):
        assert mass <= norm
        self.categorical = Categorical([norm - mass, mass])

    def norm(self):
        return self.categorical.norm()

    def pmf(self, x):
        return self.categorical.pmf(int(bool(x)))

    def cdf(self, x, i):
        return self.categorical.cdf(int(bool(x)), i)

    def icdf(self, cf):
        x, i = self.categorical.icdf(cf)
        return x != 0, i

    def push(self, m, x):
        self.categorical.push(m, int(bool(x)))

    def pop(self, m):
        return self.categorical.pop(m) != 0

    def prob(self):
        return self.categorical.prob(1)


class IID(Codec):  # src/codec.rs:405-443
    def __init__(self, item, length):
        self.item = item
        self.len = length

    def _table(self):
        if isinstance(self.item, Categorical):
            return self.item.table
        if isinstance(self.item, Bernoulli):
            return self.item.categorical.table
        return None

    def push(self, m, x):
        assert len(x) == self.len
        table = self._table()
        if table is not None:
            s = np.ascontiguousarray(np.asarray(x, dtype=np.uint32))
            _check(lib().ans_push_iid(m.h, table, _np_ptr(s), len(s)), "IID::push")
            return
        for e in reversed(list(x)):
            self.item.push(m, e)

    def pop(self, m):
        table = self._table()
        if table is not None:
            out = np.zeros(max(self.len, 1), np.uint32)
            _check(lib().ans_pop_iid(m.h, table, _np_ptr(out), self.len), "IID::pop")
            if isinstance(self.item, Bernoulli):
                return [bool(v) for v in out[:self.len]]
            return [int(v) for v in out[:self.len]]
        return [self.item.pop(m) for _ in range(self.len)]

    def bits(self, x):
        total = 0.0
        for e in x:
            b = self.item.bits(e)
            if b is None:
                return None
            total += b
        return total


class Independent(Codec):  # src/codec.rs:366-403
    def __init__(self, codecs):
        self.codecs = list(codecs)

    def push(self, m, x):
        assert len(x) == len(self.codecs)
        for c, e in reversed(list(zip(self.codecs, x))):
            c.push(m, e)

    def pop(self, m):
        return [c.pop(m) for c in self.codecs]

    def bits(self, x):
        total = 0.0
        for c, e in zip(self.codecs, x):
            b = c.bits(e)
            if b is None:
                return None
            total += b
        return total


# ============================================================== GPU bulk path (section 4)
def device_count():
    c = ci(0)
    _check(lib().ans_gpu_device_count(ctypes.byref(c)))
    return c.value


class Gpu:
    """One device context (owns a HIP stream)."""

    def __init__(self, device=0):
        h = vp()
        _check(lib().ans_gpu_create(device, ctypes.byref(h)), f"ans_gpu_create({device})")
        self.h = h
        self.device = device

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:
            _lib.ans_gpu_free(h)
            self.h = None

    def set_batch_bytes(self, batch_bytes):
        """Symbol bytes per batch of the host-buffer pipeline (0 = default, 128 MiB)."""
        _check(lib().ans_gpu_set_batch_bytes(self.h, batch_bytes), "ans_gpu_set_batch_bytes")

    def pipe_depth(self):
        """Workspace slots of the host-buffer pipeline (0 before its first call)."""
        d = ci(0)
        _check(lib().ans_gpu_pipe_depth(self.h, ctypes.byref(d)), "ans_gpu_pipe_depth")
        return d.value

    def status(self, d_status, stream=None):
        st = ci(0)
        _check(lib().ans_dev_status(self.h, _dptr(d_status), _sptr(stream), ctypes.byref(st)), "ans_dev_status")
        return st.value

    def compact(self, d_slots, slot_cap, d_lens, d_offsets, nchunks, d_out, stream=None):
        _check(lib().ans_dev_compact(self.h, _dptr(d_slots), slot_cap, _dptr(d_lens), _dptr(d_offsets), nchunks,
                                     _dptr(d_out), _sptr(stream)), "ans_dev_compact")


class _PinnedBlock:
    """Owns one ans_host_alloc block; freed when the last numpy view of it goes away."""

    def __init__(self, nbytes):
        h = vp()
        _check(lib().ans_host_alloc(max(nbytes, 1), ctypes.byref(h)), "ans_host_alloc")
        self.ptr = h.value
        self.nbytes = nbytes

    def __del__(self):
        if getattr(self, "ptr", None) and _lib is not None:
            _lib.ans_host_free(self.ptr)
            self.ptr = None


def pinned_empty(n, dtype=np.uint8):
    """A numpy array in page-locked host memory (ans_host_alloc): host-buffer GPU calls on
    it overlap their copies with the kernels."""
    dtype = np.dtype(dtype)
    blk = _PinnedBlock(n * dtype.itemsize)
    buf = (ctypes.c_char * max(n * dtype.itemsize, 1)).from_address(blk.ptr)
    buf._owner = blk  # keeps the block alive as long as any view of the buffer
    return np.frombuffer(buf, dtype=dtype, count=n)


def _dptr(t):
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def _nbytes(t):
    return t.numel() * t.element_size()


def dense_offsets_entries(nchunks):
    """u64 entries ans_dev_encode_dense needs in d_offsets for nchunks chunks."""
    return int(lib().ans_dense_offsets_entries(nchunks))


def _sptr(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


_WIDTH = {np.dtype(np.uint8): 1, np.dtype(np.uint16): 2, np.dtype(np.uint32): 4, np.dtype(np.uint64): 8}


class GpuTable:
    """A Categorical table uploaded to one device (ans_gpu_table)."""

    def __init__(self, gpu, categorical):
        self.gpu = gpu
        self.categorical = categorical
        h = vp()
        _check(lib().ans_gpu_table_create(gpu.h, categorical.table, ctypes.byref(h)), "ans_gpu_table_create")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:
            _lib.ans_gpu_table_free(h)
            self.h = None

    def paths(self):
        """ANS_PATH_* flags: which fast kernels full chunks of this table take."""
        f = ctypes.c_uint32(0)
        _check(lib().ans_gpu_table_paths(self.h, ctypes.byref(f)), "ans_gpu_table_paths")
        return f.value

    def decode_kernel(self, sym_bytes):
        """'lds' (fast::k_decode), 'global' (fast::k_decode_g) or 'generic' for full chunks."""
        p = self.paths()
        if p & ANS_PATH_DEC_LDS:
            return "lds"
        if p & ANS_PATH_DEC_WIDE and sym_bytes > 1:
            return "wide"
        if p & ANS_PATH_DEC_GLOBAL and sym_bytes > 1:
            return "global"
        return "generic"

    def slot_capacity(self, chunk_len):
        c = u64(0)
        _check(lib().ans_gpu_slot_capacity(self.h, chunk_len, ctypes.byref(c)))
        return c.value

    # ---- host buffers
    def encode_chunks(self, syms, chunk_len, gen_kind=GEN_ZEROS, seed=0):
        """syms: np array of uint8/16/32.  Returns (dense bytes, offsets u64, lens u64).  Chunk c
        starts from Message::zeros() (or Message::random(seed + c) with gen_kind=GEN_RANDOM)."""
        syms = np.ascontiguousarray(syms)
        w = _WIDTH[syms.dtype]
        n = len(syms)
        nchunks = -(-n // chunk_len)
        total = u64(0)
        # one pass into a worst-case buffer (slot capacity per chunk bounds every stream)
        out = np.empty(max(nchunks * self.slot_capacity(chunk_len), 1), np.uint8)
        offsets = np.zeros(max(nchunks, 1), np.uint64)
        lens = np.zeros(max(nchunks, 1), np.uint64)
        _check(lib().ans_gpu_encode_chunks_ex(self.h, _np_ptr(syms), w, n, chunk_len, gen_kind, seed, _np_ptr(out),
                                              len(out), _np_ptr(offsets), _np_ptr(lens), ctypes.byref(total)),
               "ans_gpu_encode_chunks")
        return out[:total.value], offsets[:nchunks], lens[:nchunks]

    def decode_chunks(self, data, offsets, lens, n, chunk_len, dtype=np.uint32, gen_kind=GEN_ZEROS, seed=0):
        data = np.ascontiguousarray(np.asarray(data, dtype=np.uint8))
        offsets = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
        lens = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
        out = np.zeros(max(n, 1), dtype)
        _check(lib().ans_gpu_decode_chunks_ex(self.h, _np_ptr(data) if data.size else None, data.size,
                                              _np_ptr(offsets), _np_ptr(lens), n, chunk_len, gen_kind, seed,
                                              _np_ptr(out), _WIDTH[np.dtype(dtype)]), "ans_gpu_decode_chunks")
        return out[:n]

    def encode_var_chunks(self, syms, starts, gen_kind=GEN_ZEROS, seed=0):
        """Variable-length chunks: chunk c = syms[starts[c]:starts[c+1]], one reference message
        each.  Returns (dense bytes, offsets u64, lens u64)."""
        syms = np.ascontiguousarray(syms)
        starts = np.ascontiguousarray(np.asarray(starts, dtype=np.uint64))
        nchunks = len(starts) - 1
        longest = int(np.diff(starts).max()) if nchunks else 0
        out = np.empty(max(nchunks * self.slot_capacity(longest), 1), np.uint8)
        offsets = np.zeros(max(nchunks, 1), np.uint64)
        lens = np.zeros(max(nchunks, 1), np.uint64)
        total = u64(0)
        _check(lib().ans_gpu_encode_var_chunks_ex(self.h, _np_ptr(syms), _WIDTH[syms.dtype], nchunks, _np_ptr(starts),
                                                  gen_kind, seed, _np_ptr(out), len(out), _np_ptr(offsets),
                                                  _np_ptr(lens), ctypes.byref(total)), "ans_gpu_encode_var_chunks")
        return out[:total.value], offsets[:nchunks], lens[:nchunks]

    def decode_var_chunks(self, data, offsets, lens, starts, dtype=np.uint32, gen_kind=GEN_ZEROS, seed=0):
        data = np.ascontiguousarray(np.asarray(data, dtype=np.uint8))
        offsets = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
        lens = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
        starts = np.ascontiguousarray(np.asarray(starts, dtype=np.uint64))
        n = int(starts[-1]) if len(starts) else 0
        out = np.zeros(max(n, 1), dtype)
        _check(lib().ans_gpu_decode_var_chunks_ex(self.h, _np_ptr(data) if data.size else None, data.size,
                                                  _np_ptr(offsets), _np_ptr(lens), len(starts) - 1, _np_ptr(starts),
                                                  gen_kind, seed, _np_ptr(out), _WIDTH[np.dtype(dtype)]),
               "ans_gpu_decode_var_chunks")
        return out[:n]

    # ---- device buffers (torch tensors or raw pointers)
    def dev_encode(self, d_syms, sym_bytes, n, chunk_len, d_slots, slot_cap, d_lens, d_status, stream=None,
                   gen_kind=GEN_ZEROS, seed=0):
        _check(lib().ans_dev_encode_chunks_ex(self.h, _dptr(d_syms), sym_bytes, n, chunk_len, gen_kind, seed,
                                              _dptr(d_slots), slot_cap, _dptr(d_lens), _dptr(d_status), _sptr(stream)),
               "ans_dev_encode_chunks")

    def dev_encode_dense(self, d_syms, sym_bytes, n, chunk_len, d_slots, slot_cap, d_lens, d_offsets, d_out,
                         d_status, stream=None, gen_kind=GEN_ZEROS, seed=0, out_cap=None):
        """Device-resident dense container (ans_dev_encode_dense_ex): d_offsets holds
        dense_offsets_entries(nchunks) u64 entries; chunk j at d_out[d_offsets[j]:][:d_lens[j]].
        out_cap: d_out's size in bytes (default: the tensor's; required for a raw pointer)."""
        if out_cap is None:
            if isinstance(d_out, int):
                raise ValueError("dev_encode_dense: out_cap is required when d_out is a raw device pointer")
            out_cap = _nbytes(d_out)
        _check(lib().ans_dev_encode_dense_ex(self.h, _dptr(d_syms), sym_bytes, n, chunk_len, gen_kind, seed,
                                             _dptr(d_slots), slot_cap, _dptr(d_lens), _dptr(d_offsets), _dptr(d_out),
                                             int(out_cap), _dptr(d_status), _sptr(stream)), "ans_dev_encode_dense")

    def dev_decode(self, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, d_syms, sym_bytes, d_status,
                   stream=None, gen_kind=GEN_ZEROS, seed=0):
        _check(lib().ans_dev_decode_chunks_ex(self.h, _dptr(d_in), _dptr(d_offsets), slot_cap, _dptr(d_lens), n,
                                              chunk_len, gen_kind, seed, _dptr(d_syms), sym_bytes, _dptr(d_status),
                                              _sptr(stream)), "ans_dev_decode_chunks")

    def sample_chunks(self, seed, n, chunk_len, dtype=np.uint32):
        """Codec::samples in bulk (src/ans.rs:42-44): chunk c = samples(len, seed + c)."""
        out = np.zeros(max(n, 1), dtype)
        _check(lib().ans_gpu_sample_iid(self.h, seed, n, chunk_len, _np_ptr(out), _WIDTH[np.dtype(dtype)]),
               "ans_gpu_sample_iid")
        return out[:n]

    def dev_sample(self, seed, n, chunk_len, d_syms, sym_bytes, stream=None):
        _check(lib().ans_dev_sample_iid(self.h, seed, n, chunk_len, _dptr(d_syms), sym_bytes, _sptr(stream)),
               "ans_dev_sample_iid")

    def dev_gen_iid(self, seed, start, n, d_syms, sym_bytes, stream=None):
        _check(lib().ans_dev_gen_iid(self.h, seed, start, n, _dptr(d_syms), sym_bytes, _sptr(stream)),
               "ans_dev_gen_iid")


# ============================================================== other static codecs (section 4b)
def _enc_buffers(n, chunk_len, per_symbol=8):
    nchunks = -(-n // chunk_len)
    out = np.empty(max(per_symbol * n + 16 * nchunks + 64, 1), np.uint8)
    return nchunks, out, np.zeros(max(nchunks, 1), np.uint64), np.zeros(max(nchunks, 1), np.uint64)


def _dec_arrays(data, offsets, lens):
    data = np.ascontiguousarray(np.asarray(data, dtype=np.uint8))
    return (data, np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64)),
            np.ascontiguousarray(np.asarray(lens, dtype=np.uint64)))


class GpuUniform:
    """IID<Uniform(size)> in chunks on the GPU (src/codec.rs:13-49; size <= 2^46)."""

    def __init__(self, gpu, size):
        self.gpu, self.size = gpu, int(size)

    def encode_chunks(self, syms, chunk_len, gen_kind=GEN_ZEROS, seed=0):
        syms = np.ascontiguousarray(syms)
        n = len(syms)
        nchunks, out, offsets, lens = _enc_buffers(n, chunk_len)
        total = u64(0)
        _check(lib().ans_gpu_uniform_encode_chunks(self.gpu.h, self.size, _np_ptr(syms), _WIDTH[syms.dtype], n,
                                                   chunk_len, gen_kind, seed, _np_ptr(out), len(out), _np_ptr(offsets),
                                                   _np_ptr(lens), ctypes.byref(total)), "ans_gpu_uniform_encode_chunks")
        return out[:total.value], offsets[:nchunks], lens[:nchunks]

    def decode_chunks(self, data, offsets, lens, n, chunk_len, dtype=np.uint64, gen_kind=GEN_ZEROS, seed=0):
        data, offsets, lens = _dec_arrays(data, offsets, lens)
        out = np.zeros(max(n, 1), dtype)
        _check(lib().ans_gpu_uniform_decode_chunks(self.gpu.h, self.size, _np_ptr(data) if data.size else None,
                                                   data.size, _np_ptr(offsets), _np_ptr(lens), n, chunk_len, gen_kind,
                                                   seed, _np_ptr(out), _WIDTH[np.dtype(dtype)]),
               "ans_gpu_uniform_decode_chunks")
        return out[:n]


    # device-resident (include/ans_capi.h 4b): fixed chunks in slots, asynchronous on `stream`
    def slot_capacity(self, chunk_len):
        c = u64(0)
        _check(lib().ans_gpu_uniform_slot_capacity(self.size, chunk_len, ctypes.byref(c)), "ans_gpu_uniform_slot_capacity")
        return c.value

    def dev_encode(self, d_syms, sym_bytes, n, chunk_len, d_slots, slot_cap, d_lens, d_status, stream=None,
                   gen_kind=GEN_ZEROS, seed=0):
        _check(lib().ans_dev_uniform_encode(self.gpu.h, self.size, _dptr(d_syms), sym_bytes, n, chunk_len, gen_kind, seed,
                                            _dptr(d_slots), slot_cap, _dptr(d_lens), _dptr(d_status), _sptr(stream)),
               "ans_dev_uniform_encode")

    def dev_decode(self, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, d_syms, sym_bytes, d_status, stream=None,
                   gen_kind=GEN_ZEROS, seed=0):
        _check(lib().ans_dev_uniform_decode(self.gpu.h, self.size, _dptr(d_in), _dptr(d_offsets), slot_cap,
                                            _dptr(d_lens), n, chunk_len, gen_kind, seed, _dptr(d_syms), sym_bytes,
                                            _dptr(d_status), _sptr(stream)), "ans_dev_uniform_decode")


class GpuLogUniform:
    """IID<LogUniform::new(excl_max_bits)> in chunks on the GPU (src/codec.rs:561-611), the item
    of MaxBenfordIID (src/param_codec.rs:117-119)."""

    def __init__(self, gpu, excl_max_bits):
        self.gpu, self.excl_max_bits = gpu, int(excl_max_bits)

    def encode_chunks(self, syms, chunk_len, gen_kind=GEN_ZEROS, seed=0):
        syms = np.ascontiguousarray(syms)
        n = len(syms)
        nchunks, out, offsets, lens = _enc_buffers(n, chunk_len)
        total = u64(0)
        _check(lib().ans_gpu_loguniform_encode_chunks(self.gpu.h, self.excl_max_bits, _np_ptr(syms), _WIDTH[syms.dtype],
                                                      n, chunk_len, gen_kind, seed, _np_ptr(out), len(out),
                                                      _np_ptr(offsets), _np_ptr(lens), ctypes.byref(total)),
               "ans_gpu_loguniform_encode_chunks")
        return out[:total.value], offsets[:nchunks], lens[:nchunks]

    def decode_chunks(self, data, offsets, lens, n, chunk_len, dtype=np.uint64, gen_kind=GEN_ZEROS, seed=0):
        data, offsets, lens = _dec_arrays(data, offsets, lens)
        out = np.zeros(max(n, 1), dtype)
        _check(lib().ans_gpu_loguniform_decode_chunks(self.gpu.h, self.excl_max_bits,
                                                      _np_ptr(data) if data.size else None, data.size,
                                                      _np_ptr(offsets), _np_ptr(lens), n, chunk_len, gen_kind, seed,
                                                      _np_ptr(out), _WIDTH[np.dtype(dtype)]),
               "ans_gpu_loguniform_decode_chunks")
        return out[:n]


    def slot_capacity(self, chunk_len):
        c = u64(0)
        _check(lib().ans_gpu_loguniform_slot_capacity(self.excl_max_bits, chunk_len, ctypes.byref(c)),
               "ans_gpu_loguniform_slot_capacity")
        return c.value

    def dev_encode(self, d_syms, sym_bytes, n, chunk_len, d_slots, slot_cap, d_lens, d_status, stream=None,
                   gen_kind=GEN_ZEROS, seed=0):
        _check(lib().ans_dev_loguniform_encode(self.gpu.h, self.excl_max_bits, _dptr(d_syms), sym_bytes, n, chunk_len,
                                               gen_kind, seed, _dptr(d_slots), slot_cap, _dptr(d_lens), _dptr(d_status),
                                               _sptr(stream)), "ans_dev_loguniform_encode")

    def dev_decode(self, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, d_syms, sym_bytes, d_status, stream=None,
                   gen_kind=GEN_ZEROS, seed=0):
        _check(lib().ans_dev_loguniform_decode(self.gpu.h, self.excl_max_bits, _dptr(d_in), _dptr(d_offsets), slot_cap,
                                               _dptr(d_lens), n, chunk_len, gen_kind, seed, _dptr(d_syms), sym_bytes,
                                               _dptr(d_status), _sptr(stream)), "ans_dev_loguniform_decode")


class GpuTableSet:
    """Independent<Categorical> (src/codec.rs:366-403) on the GPU: a set of Categoricals uploaded
    once; position k codes with table table_ids[k]."""

    def __init__(self, gpu, categoricals):
        self.gpu = gpu
        self.categoricals = list(categoricals)
        arr = (vp * len(self.categoricals))(*[c.table for c in self.categoricals])
        h = vp()
        _check(lib().ans_gpu_tableset_create(gpu.h, arr, len(self.categoricals), ctypes.byref(h)),
               "ans_gpu_tableset_create")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h and _lib is not None:
            _lib.ans_gpu_tableset_free(h)
            self.h = None

    def encode_chunks(self, table_ids, syms, chunk_len, gen_kind=GEN_ZEROS, seed=0):
        syms = np.ascontiguousarray(syms)
        tids = np.ascontiguousarray(np.asarray(table_ids, dtype=np.uint32))
        n = len(syms)
        nchunks, out, offsets, lens = _enc_buffers(n, chunk_len)
        total = u64(0)
        _check(lib().ans_gpu_independent_encode_chunks(self.h, _np_ptr(tids), _np_ptr(syms), _WIDTH[syms.dtype], n,
                                                       chunk_len, gen_kind, seed, _np_ptr(out), len(out),
                                                       _np_ptr(offsets), _np_ptr(lens), ctypes.byref(total)),
               "ans_gpu_independent_encode_chunks")
        return out[:total.value], offsets[:nchunks], lens[:nchunks]

    def decode_chunks(self, table_ids, data, offsets, lens, chunk_len, dtype=np.uint32, gen_kind=GEN_ZEROS, seed=0):
        data, offsets, lens = _dec_arrays(data, offsets, lens)
        tids = np.ascontiguousarray(np.asarray(table_ids, dtype=np.uint32))
        n = len(tids)
        out = np.zeros(max(n, 1), dtype)
        _check(lib().ans_gpu_independent_decode_chunks(self.h, _np_ptr(tids), _np_ptr(data) if data.size else None,
                                                       data.size, _np_ptr(offsets), _np_ptr(lens), n, chunk_len,
                                                       gen_kind, seed, _np_ptr(out), _WIDTH[np.dtype(dtype)]),
               "ans_gpu_independent_decode_chunks")
        return out[:n]

    def encode_var_chunks(self, table_ids, syms, starts, gen_kind=GEN_ZEROS, seed=0):
        """Chunk c = positions [starts[c], starts[c+1]), one message each (the exact kernels)."""
        syms = np.ascontiguousarray(syms)
        tids = np.ascontiguousarray(np.asarray(table_ids, dtype=np.uint32))
        st = np.ascontiguousarray(np.asarray(starts, dtype=np.uint64))
        nchunks = len(st) - 1
        longest = int(np.max(np.diff(st))) if nchunks else 0
        cap = max(nchunks * self.slot_capacity(max(longest, 1)), 1)
        out = np.empty(cap, np.uint8)
        offsets = np.zeros(max(nchunks, 1), np.uint64)
        lens = np.zeros(max(nchunks, 1), np.uint64)
        total = u64(0)
        _check(lib().ans_gpu_independent_encode_var_chunks(self.h, _np_ptr(tids), _np_ptr(syms), _WIDTH[syms.dtype],
                                                           nchunks, _np_ptr(st), gen_kind, seed, _np_ptr(out), cap,
                                                           _np_ptr(offsets), _np_ptr(lens), ctypes.byref(total)),
               "ans_gpu_independent_encode_var_chunks")
        return out[:total.value], offsets[:nchunks], lens[:nchunks]

    def decode_var_chunks(self, table_ids, data, offsets, lens, starts, dtype=np.uint32, gen_kind=GEN_ZEROS, seed=0):
        data, offsets, lens = _dec_arrays(data, offsets, lens)
        tids = np.ascontiguousarray(np.asarray(table_ids, dtype=np.uint32))
        st = np.ascontiguousarray(np.asarray(starts, dtype=np.uint64))
        nchunks = len(st) - 1
        n = int(st[-1]) if nchunks else 0
        out = np.zeros(max(n, 1), dtype)
        _check(lib().ans_gpu_independent_decode_var_chunks(self.h, _np_ptr(tids), _np_ptr(data) if data.size else None,
                                                           data.size, _np_ptr(offsets), _np_ptr(lens), nchunks,
                                                           _np_ptr(st), gen_kind, seed, _np_ptr(out),
                                                           _WIDTH[np.dtype(dtype)]),
               "ans_gpu_independent_decode_var_chunks")
        return out[:n]

    def fast(self):
        """1 / 2: the set runs on the fast kernels (2: with voted exact renorm rows); 0: exact only."""
        f = ci(0)
        _check(lib().ans_gpu_tableset_fast(self.h, ctypes.byref(f)), "ans_gpu_tableset_fast")
        return f.value

    def lanes(self, lanes):
        """The fast kernels' workgroup layout: 0 by call size, 256, or 1024 (one shared table image)."""
        _check(lib().ans_gpu_tableset_lanes(self.h, lanes), "ans_gpu_tableset_lanes")

    def slot_capacity(self, chunk_len):
        c = u64(0)
        _check(lib().ans_gpu_tableset_slot_capacity(self.h, chunk_len, ctypes.byref(c)), "ans_gpu_tableset_slot_capacity")
        return c.value

    def dev_encode(self, d_tids, d_syms, sym_bytes, n, chunk_len, d_slots, slot_cap, d_lens, d_status, stream=None,
                   gen_kind=GEN_ZEROS, seed=0):
        """d_tids: one byte per position (device)."""
        _check(lib().ans_dev_independent_encode(self.h, _dptr(d_tids), _dptr(d_syms), sym_bytes, n, chunk_len, gen_kind,
                                                seed, _dptr(d_slots), slot_cap, _dptr(d_lens), _dptr(d_status),
                                                _sptr(stream)), "ans_dev_independent_encode")

    def dev_decode(self, d_tids, d_in, d_offsets, slot_cap, d_lens, n, chunk_len, d_syms, sym_bytes, d_status,
                   stream=None, gen_kind=GEN_ZEROS, seed=0):
        _check(lib().ans_dev_independent_decode(self.h, _dptr(d_tids), _dptr(d_in), _dptr(d_offsets), slot_cap,
                                                _dptr(d_lens), n, chunk_len, gen_kind, seed, _dptr(d_syms), sym_bytes,
                                                _dptr(d_status), _sptr(stream)), "ans_dev_independent_decode")


# ============================================================== graph models' bulk caller (section 5)
class AllEdgeIndices:
    """The edge alphabet of src/graph_codec.rs:176-205 in the reference's order: the
    self-loops (i, i) first when allowed, then for j in 0..n, i in 0..j the pair (i, j),
    followed by (j, i) when directed."""

    def __init__(self, num_nodes, directed=False, loops=False):
        self.num_nodes, self.directed, self.loops = int(num_nodes), bool(directed), bool(loops)

    def __len__(self):  # num_all_edge_indices, src/graph_codec.rs:203-205
        n = u64(0)
        _check(lib().ans_edge_alphabet_len(self.num_nodes, int(self.directed), int(self.loops), ctypes.byref(n)),
               "num_all_edge_indices")
        return n.value

    def __iter__(self):
        n = self.num_nodes
        if self.loops:
            for i in range(n):
                yield (i, i)
        for j in range(n):
            for i in range(j):
                yield (i, j)
                if self.directed:
                    yield (j, i)


class DenseSetIID(Codec):
    """src/graph_codec.rs:104-139: a set over `alphabet` coded as IID<Bernoulli> of its
    indicator vector, on ONE message (the reference's bitstream)."""

    def __init__(self, contains, alphabet):
        self.alphabet = alphabet
        self.contains = IID(contains, len(alphabet))

    def dense(self, x):  # src/graph_codec.rs:133-138
        rest = set(map(tuple, x))
        out = []
        for a in self.alphabet:
            out.append(a in rest)
            rest.discard(a)
        if rest:
            raise AnsError(ANS_E_SYMBOL, "DenseSetIID::dense: element outside the alphabet")
        return out

    def push(self, m, x):
        self.contains.push(m, self.dense(x))

    def pop(self, m):
        d = self.contains.pop(m)
        return [a for a, b in zip(self.alphabet, d) if b]

    def bits(self, x):
        return self.contains.bits(self.dense(x))


class ErdosRenyi(DenseSetIID):
    """erdos_renyi_indices (src/graph_codec.rs:172-174): DenseSetIID over AllEdgeIndices."""

    def __init__(self, edge, num_nodes, directed=False, loops=False):
        super().__init__(edge, AllEdgeIndices(num_nodes, directed, loops))
        self.loops = loops


class GpuDenseSet:
    """The ErdosRenyi edge set on the GPU (section 5 of the C ABI): the dense indicator
    vector is built on the device, coded by the bulk chunk path with the Bernoulli table and
    decoded back to the edge list in alphabet order.  Chunk j is one reference message over
    alphabet slots [j*chunk_len, (j+1)*chunk_len)."""

    def __init__(self, gpu, edge, num_nodes, directed=False, loops=False):
        self.gpu = gpu
        self.edge = edge
        self.table = GpuTable(gpu, edge.categorical)
        self.space = (int(num_nodes), int(bool(directed)), int(bool(loops)))

    def alphabet_len(self):
        return len(AllEdgeIndices(*self.space))

    def encode(self, edges, chunk_len):
        """edges: (m, 2) integer array of (i, j).  Returns (bytes, offsets, lens)."""
        e = np.ascontiguousarray(np.asarray(edges, dtype=np.uint32).reshape(-1, 2))
        n = self.alphabet_len()
        nchunks = -(-n // chunk_len)
        out = np.empty(max(nchunks * self.table.slot_capacity(chunk_len), 1), np.uint8)
        offsets = np.zeros(max(nchunks, 1), np.uint64)
        lens = np.zeros(max(nchunks, 1), np.uint64)
        total = u64(0)
        _check(lib().ans_gpu_dense_set_encode(self.table.h, *self.space, _np_ptr(e), len(e), chunk_len, _np_ptr(out),
                                              len(out), _np_ptr(offsets), _np_ptr(lens), ctypes.byref(total)),
               "ans_gpu_dense_set_encode")
        return out[:total.value], offsets[:nchunks], lens[:nchunks]

    def decode(self, data, offsets, lens, chunk_len, cap=None):
        data = np.ascontiguousarray(np.asarray(data, dtype=np.uint8))
        offsets = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
        lens = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
        if cap is None:  # the expected edge count with room; a second pass if it is exceeded
            cap = int(2 * self.edge.prob() * self.alphabet_len()) + 1024
        cap = min(cap, self.alphabet_len())
        for _ in range(2):
            edges = np.zeros((max(cap, 1), 2), np.uint32)
            count = u64(0)
            rc = lib().ans_gpu_dense_set_decode(self.table.h, *self.space, _np_ptr(data) if data.size else None,
                                                data.size, _np_ptr(offsets), _np_ptr(lens), chunk_len, _np_ptr(edges),
                                                cap, ctypes.byref(count))
            if rc == ANS_E_LEN and count.value > cap:
                cap = count.value
                continue
            _check(rc, "ans_gpu_dense_set_decode")
            return edges[:count.value]
        raise AnsError(ANS_E_LEN, "ans_gpu_dense_set_decode")


class GpuDenseSets:
    """A dataset of graphs under one ErdosRenyi Bernoulli (GraphDatasetParamCodec with
    ErdosRenyiParamCodec, src/param_codec.rs:171-199,243-293) on the GPU: graph g is one
    message (one chunk of the variable-chunk path)."""

    def __init__(self, gpu, edge, directed=False, loops=False):
        self.gpu = gpu
        self.edge = edge
        self.table = GpuTable(gpu, edge.categorical)
        self.directed, self.loops = int(bool(directed)), int(bool(loops))

    def encode(self, num_nodes, edge_lists):
        """num_nodes: per graph; edge_lists: per graph an (m_g, 2) array.  Returns
        (bytes, offsets, lens), one stream per graph."""
        nn = np.ascontiguousarray(np.asarray(num_nodes, dtype=np.uint32))
        parts = [np.asarray(e, dtype=np.uint32).reshape(-1, 2) for e in edge_lists]
        eo = np.zeros(len(parts) + 1, np.uint64)
        eo[1:] = np.cumsum([len(p) for p in parts])
        edges = np.ascontiguousarray(np.concatenate(parts) if parts else np.zeros((0, 2), np.uint32))
        sizes = [len(AllEdgeIndices(int(n), self.directed, self.loops)) for n in nn]
        cap = sum(self.table.slot_capacity(max(sizes) if sizes else 0) for _ in sizes)
        out = np.empty(max(cap, 1), np.uint8)
        offsets = np.zeros(max(len(nn), 1), np.uint64)
        lens = np.zeros(max(len(nn), 1), np.uint64)
        total = u64(0)
        _check(lib().ans_gpu_dense_sets_encode(self.table.h, len(nn), _np_ptr(nn), self.directed, self.loops,
                                               _np_ptr(edges), _np_ptr(eo), _np_ptr(out), len(out), _np_ptr(offsets),
                                               _np_ptr(lens), ctypes.byref(total)), "ans_gpu_dense_sets_encode")
        return out[:total.value], offsets[:len(nn)], lens[:len(nn)]

    def decode(self, num_nodes, data, offsets, lens, cap=None):
        """Returns the per-graph edge arrays (alphabet order)."""
        nn = np.ascontiguousarray(np.asarray(num_nodes, dtype=np.uint32))
        data = np.ascontiguousarray(np.asarray(data, dtype=np.uint8))
        offsets = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
        lens = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
        slots = sum(len(AllEdgeIndices(int(n), self.directed, self.loops)) for n in nn)
        if cap is None:
            cap = int(2 * self.edge.prob() * slots) + 1024
        cap = min(cap, slots)
        eo = np.zeros(len(nn) + 1, np.uint64)
        for _ in range(2):
            edges = np.zeros((max(cap, 1), 2), np.uint32)
            rc = lib().ans_gpu_dense_sets_decode(self.table.h, len(nn), _np_ptr(nn), self.directed, self.loops,
                                                 _np_ptr(data) if data.size else None, data.size, _np_ptr(offsets),
                                                 _np_ptr(lens), _np_ptr(edges), cap, _np_ptr(eo))
            if rc == ANS_E_LEN and int(eo[-1]) > cap:
                cap = int(eo[-1])
                continue
            _check(rc, "ans_gpu_dense_sets_decode")
            return [edges[int(eo[g]):int(eo[g + 1])] for g in range(len(nn))]
        raise AnsError(ANS_E_LEN, "ans_gpu_dense_sets_decode")


class EmptyCodec(Codec):
    """ConstantCodec<()> (src/codec.rs, graph_codec.rs:16 EmptyCodec): codes nothing."""

    def push(self, m, x):
        pass

    def pop(self, m):
        return None

    def bits(self, x):
        return 0.0


class Graph(collections.namedtuple("Graph", "node_labels edges")):
    """Graph<N, E, Ty> as GraphIID codes it (src/graph.rs:89-168): node_labels (one per node;
    None entries for EmptyCodec nodes) and edges, a list of ((i, j), label) (label None for
    unlabelled edges; undirected pairs have i <= j)."""

    def __len__(self):
        return len(self.node_labels)


class EdgesIID(Codec):  # src/graph_codec.rs:51-94
    def __init__(self, indices, label=None):
        self.indices = indices
        self.label = label if label is not None else EmptyCodec()

    @staticmethod
    def split(x):  # src/graph_codec.rs:82-85: sorted by the edge index (a tuple)
        s = sorted(((tuple(map(int, i)), l) for i, l in x), key=lambda e: e[0])
        return [e[0] for e in s], [e[1] for e in s]

    def push(self, m, x):  # src/graph_codec.rs:61-65
        indices, labels = self.split(x)
        IID(self.label, len(indices)).push(m, labels)
        self.indices.push(m, indices)

    def pop(self, m):  # src/graph_codec.rs:67-71
        indices = sorted(self.indices.pop(m))
        labels = IID(self.label, len(indices)).pop(m)
        return list(zip(indices, labels))

    def bits(self, x):
        indices, labels = self.split(x)
        a, b = self.indices.bits(indices), IID(self.label, len(indices)).bits(labels)
        return None if a is None or b is None else a + b


class GraphIID(Codec):  # src/graph_codec.rs:19-49
    """GraphIID::new(num_nodes, edge_indices, node, edge): the node labels IID, the edges through
    EdgesIID; None for node / edge is EmptyCodec."""

    def __init__(self, num_nodes, edge_indices, node=None, edge=None):
        self.nodes = IID(node if node is not None else EmptyCodec(), num_nodes)
        self.edges = EdgesIID(edge_indices, edge)

    def push(self, m, x):  # src/graph_codec.rs:31-34
        self.edges.push(m, x.edges)
        self.nodes.push(m, list(x.node_labels))

    def pop(self, m):  # src/graph_codec.rs:36-38
        nodes = self.nodes.pop(m)
        return Graph(nodes, self.edges.pop(m))

    def bits(self, x):
        a, b = self.nodes.bits(list(x.node_labels)), self.edges.bits(x.edges)
        return None if a is None or b is None else a + b


def _label_categorical(c):
    """A label codec as the Categorical the GPU table set holds: Uniform(size) becomes the all-ones
    Categorical of that size (pmf 1, cdf x, norm size: Uniform's arithmetic)."""
    if c is None or isinstance(c, EmptyCodec):
        return None
    if isinstance(c, Categorical):
        return c
    if isinstance(c, Uniform):
        return Categorical(np.ones(c.size, np.uint64))
    raise TypeError(f"no GPU table for {type(c).__name__}")


class GpuGraphs:
    """Independent<GraphIID<NodeC, EdgeC, ErdosRenyi>> over a dataset on the GPU (section 5b of
    the C ABI): every graph's message is GraphIID::push of that graph on Message::zeros(), with one
    Bernoulli for the edge indicators and Categorical (or Uniform) node / edge labels, as the
    reference's --er / --uniform-er models build them (src/benchmark.rs:308-372)."""

    def __init__(self, gpu, edge, node=None, edge_label=None, directed=False, loops=False):
        self.gpu = gpu
        self.edge = edge
        self.node_cat, self.edge_cat = _label_categorical(node), _label_categorical(edge_label)
        tables = [edge.categorical] + [c for c in (self.node_cat, self.edge_cat) if c is not None]
        self.tableset = GpuTableSet(gpu, tables)
        self.t_node = 1 if self.node_cat is not None else ANS_NO_TABLE
        self.t_edge = (2 if self.node_cat is not None else 1) if self.edge_cat is not None else ANS_NO_TABLE
        self.directed, self.loops = int(bool(directed)), int(bool(loops))

    def fast(self):
        return self.tableset.fast()

    def _sizes(self, num_nodes):
        return [len(AllEdgeIndices(int(n), self.directed, self.loops)) for n in num_nodes]

    def encode(self, graphs, gen_kind=GEN_ZEROS, seed=0):
        """graphs: per graph (num_nodes, node_labels or None, edges (m, 2), edge_labels or None).
        Returns (bytes, offsets, lens), one stream per graph."""
        nn = np.ascontiguousarray(np.asarray([int(g[0]) for g in graphs], dtype=np.uint32))
        nl = [np.asarray(g[1] if g[1] is not None else np.zeros(0), dtype=np.uint32).reshape(-1) for g in graphs]
        parts = [np.asarray(g[2], dtype=np.uint32).reshape(-1, 2) for g in graphs]
        el = [np.asarray(g[3] if g[3] is not None else np.zeros(0), dtype=np.uint32).reshape(-1) for g in graphs]
        eo = np.zeros(len(parts) + 1, np.uint64)
        eo[1:] = np.cumsum([len(p) for p in parts])
        edges = np.ascontiguousarray(np.concatenate(parts) if parts else np.zeros((0, 2), np.uint32))
        node_labels = np.ascontiguousarray(np.concatenate(nl) if nl else np.zeros(0, np.uint32))
        edge_labels = np.ascontiguousarray(np.concatenate(el) if el else np.zeros(0, np.uint32))
        sizes = self._sizes(nn)
        longest = max([int(n) + s + len(p) for n, s, p in zip(nn, sizes, parts)] + [1])
        cap = max(len(nn) * self.tableset.slot_capacity(longest), 1)
        out = np.empty(cap, np.uint8)
        offsets = np.zeros(max(len(nn), 1), np.uint64)
        lens = np.zeros(max(len(nn), 1), np.uint64)
        total = u64(0)
        _check(lib().ans_gpu_graphs_encode(self.tableset.h, self.t_node, self.t_edge, 0, self.directed, self.loops,
                                           len(nn), _np_ptr(nn), _np_ptr(node_labels) if node_labels.size else None,
                                           _np_ptr(edges), _np_ptr(edge_labels) if edge_labels.size else None,
                                           _np_ptr(eo), gen_kind, seed, _np_ptr(out), cap, _np_ptr(offsets),
                                           _np_ptr(lens), ctypes.byref(total)), "ans_gpu_graphs_encode")
        return out[:total.value], offsets[:len(nn)], lens[:len(nn)]

    def decode(self, num_nodes, data, offsets, lens, cap=None, gen_kind=GEN_ZEROS, seed=0):
        """Per graph (node_labels or None, edges sorted by (i, j), edge_labels or None)."""
        nn = np.ascontiguousarray(np.asarray(num_nodes, dtype=np.uint32))
        data, offsets, lens = _dec_arrays(data, offsets, lens)
        slots = sum(self._sizes(nn))
        if cap is None:
            cap = int(2 * self.edge.prob() * slots) + 1024
        cap = min(cap, slots)
        node_labels = np.zeros(max(int(nn.sum()), 1), np.uint32)
        eo = np.zeros(len(nn) + 1, np.uint64)
        for _ in range(2):
            edges = np.zeros((max(cap, 1), 2), np.uint32)
            edge_labels = np.zeros(max(cap, 1), np.uint32)
            rc = lib().ans_gpu_graphs_decode(self.tableset.h, self.t_node, self.t_edge, 0, self.directed, self.loops,
                                             len(nn), _np_ptr(nn), _np_ptr(data) if data.size else None, data.size,
                                             _np_ptr(offsets), _np_ptr(lens), gen_kind, seed, _np_ptr(node_labels),
                                             _np_ptr(edges), _np_ptr(edge_labels), cap, _np_ptr(eo))
            if rc == ANS_E_LEN and int(eo[-1]) > cap:
                cap = int(eo[-1])
                continue
            _check(rc, "ans_gpu_graphs_decode")
            no = np.concatenate([[0], np.cumsum(nn.astype(np.uint64))]).astype(np.int64)
            out = []
            for g in range(len(nn)):
                a, b = int(eo[g]), int(eo[g + 1])
                out.append((node_labels[no[g]:no[g + 1]].copy() if self.node_cat is not None else None,
                            edges[a:b].copy(), edge_labels[a:b].copy() if self.edge_cat is not None else None))
            return out
        raise AnsError(ANS_E_LEN, "ans_gpu_graphs_decode")


# ============================================================== synthetic tables
def splitmix64_np(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def c3_masses():
    """256 masses 1 + (splitmix64(0x5EED ^ s) mod 2^20): norm 139,224,331."""
    s = np.arange(256, dtype=np.uint64)
    return (np.uint64(1) + (splitmix64_np(np.uint64(0x5EED) ^ s) & np.uint64((1 << 20) - 1))).astype(np.uint64)


def quantise_masses(m, target):
    """Largest-remainder rounding of masses m to sum exactly `target`, every mass at least 1."""
    m = np.asarray(m, dtype=np.float64)
    exact = m * target / m.sum()
    q = np.maximum(1, np.floor(exact)).astype(np.int64)
    rem = target - int(q.sum())
    order = np.argsort(-(exact - np.floor(exact)))
    i = 0
    while rem != 0:
        k = order[i % len(order)]
        if rem > 0:
            q[k] += 1
            rem -= 1
        elif q[k] > 1:
            q[k] -= 1
            rem += 1
        i += 1
    return q.astype(np.uint64)


def c3_pow2_masses():
    """C3's table quantised to norm 2^24 (SURVEY.md §8d secondary C3)."""
    return quantise_masses(c3_masses(), 1 << 24)


def c3_small_masses():
    """C3's table quantised to norm 32,749 (a prime below 2^15): the norm range of the
    reference's dataset-level tables built from counts (src/benchmark.rs:552-578)."""
    return quantise_masses(c3_masses(), 32749)


def c3_big_masses():
    """C3's table quantised to norm 4,294,967,291 (the largest prime below 2^32)."""
    return quantise_masses(c3_masses(), 4294967291)


def c4_masses():
    """65,536 masses 1 + (splitmix64(0xC4 ^ s) mod 2^12): norm 134,561,356."""
    s = np.arange(65536, dtype=np.uint64)
    return (np.uint64(1) + (splitmix64_np(np.uint64(0xC4) ^ s) & np.uint64((1 << 12) - 1))).astype(np.uint64)


def c4_small_masses():
    """The first 4,096 of C4's masses quantised to norm 65,521 (the largest prime below 2^16): a
    large-alphabet table in the count-built norm range (src/benchmark.rs:576-578)."""
    return quantise_masses(c4_masses()[:4096], 65521)


def c4_big_masses():
    """C4's 65,536 masses quantised to norm 4,294,967,291 (the largest prime below 2^32)."""
    return quantise_masses(c4_masses(), 4294967291)


def read_multiset(path):
    """The reference harness' reader (src/multiset.rs:161-166): ", "-separated integers."""
    with open(path) as f:
        return [int(s) for s in f.read().split(", ")]


def multiset_masses(probs, norm=1 << 28):
    """max(1, (p * norm) as usize) (src/multiset.rs:169-170)."""
    return [max(1, int(p * float(norm))) for p in probs]
