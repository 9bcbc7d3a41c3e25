"""ctypes wrapper around oracle/build/libans_oracle.so (the C restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — as the checker, never as the product path.
See oracle/ans_oracle.c for what it restates (src/ans.rs, src/codec.rs).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libans_oracle.so")

ZEROS, EMPTY, RANDOM = 0, 1, 2
_lib = None

u64 = ctypes.c_uint64
u32 = ctypes.c_uint32
vp = ctypes.c_void_p


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        sigs = {
            "orc_msg_new": (vp, [ctypes.c_int, u64]),
            "orc_msg_free": (None, [vp]),
            "orc_msg_clone": (vp, [vp]),
            "orc_msg_err": (ctypes.c_int, [vp]),
            "orc_msg_head": (u64, [vp]),
            "orc_msg_tail_len": (u64, [vp]),
            "orc_msg_num_generated": (u64, [vp]),
            "orc_msg_flatten": (u64, [vp, vp, u64]),
            "orc_msg_unflatten": (vp, [vp, u64, ctypes.c_int, u64]),
            "orc_msg_reflatten": (vp, [vp]),
            "orc_msg_bits": (u64, [vp]),
            "orc_msg_virtual_bits": (ctypes.c_double, [vp]),
            "orc_msg_equal": (ctypes.c_int, [vp, vp]),
            "orc_cat_new": (vp, [vp, u32]),
            "orc_cat_free": (None, [vp]),
            "orc_cat_norm": (u64, [vp]),
            "orc_cat_push": (ctypes.c_int, [vp, vp, u64]),
            "orc_cat_pop": (ctypes.c_int, [vp, vp, ctypes.POINTER(u64)]),
            "orc_uniform_push": (ctypes.c_int, [vp, u64, u64]),
            "orc_uniform_pop": (ctypes.c_int, [vp, u64, ctypes.POINTER(u64)]),
            "orc_iid_push": (ctypes.c_int, [vp, vp, vp, u64]),
            "orc_iid_pop": (ctypes.c_int, [vp, vp, vp, u64]),
            "orc_encode_chunks": (ctypes.c_int, [vp, u32, vp, u64, u64, ctypes.c_int, u64, vp, u64, vp, vp]),
            "orc_decode_chunks": (ctypes.c_int, [vp, u32, vp, vp, vp, u64, u64, ctypes.c_int, u64, vp]),
            "orc_gen_iid": (ctypes.c_int, [vp, u32, u64, u64, u64, vp]),
            "orc_splitmix64": (u64, [u64]),
            "orc_codec_encode_chunks": (ctypes.c_int, [ctypes.c_int, u64, u32, vp, vp, vp, vp, u64, u64, ctypes.c_int,
                                                       u64, vp, u64, vp, vp]),
            "orc_codec_decode_chunks": (ctypes.c_int, [ctypes.c_int, u64, u32, vp, vp, vp, vp, vp, vp, u64, u64,
                                                       ctypes.c_int, u64, vp]),
        }
        for name, (res, args) in sigs.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Message:
    """Mirror of the reference `Message` (src/ans.rs:225-310) backed by the C oracle."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def zeros(cls):
        return cls(lib().orc_msg_new(ZEROS, 0))

    @classmethod
    def empty(cls):
        return cls(lib().orc_msg_new(EMPTY, 0))

    @classmethod
    def random(cls, seed):
        return cls(lib().orc_msg_new(RANDOM, seed))

    @classmethod
    def unflatten(cls, data, kind=ZEROS, seed=0):
        buf = np.frombuffer(bytes(data), dtype=np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        return cls(lib().orc_msg_unflatten(_ptr(buf), len(data), kind, seed))

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_msg_free(self.h)
            self.h = None

    def clone(self):
        return Message(lib().orc_msg_clone(self.h))

    @property
    def head(self):
        return lib().orc_msg_head(self.h)

    @property
    def err(self):
        return lib().orc_msg_err(self.h)

    @property
    def num_generated(self):
        return lib().orc_msg_num_generated(self.h)

    def flatten(self):
        n = lib().orc_msg_flatten(self.h, None, 0)
        buf = np.zeros(max(n, 1), np.uint8)
        lib().orc_msg_flatten(self.h, _ptr(buf), n)
        return bytes(buf[:n])

    def reflatten(self):
        return Message(lib().orc_msg_reflatten(self.h))

    def bits(self):
        return lib().orc_msg_bits(self.h)

    def virtual_bits(self):
        return lib().orc_msg_virtual_bits(self.h)

    def __eq__(self, other):
        return bool(lib().orc_msg_equal(self.h, other.h))


class Categorical:
    """Mirror of `Categorical` (src/codec.rs:51-92) backed by the C oracle."""

    def __init__(self, masses):
        self.masses = np.ascontiguousarray(np.asarray(masses, dtype=np.uint64))
        self.h = lib().orc_cat_new(_ptr(self.masses), len(self.masses))

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_cat_free(self.h)
            self.h = None

    @property
    def norm(self):
        return lib().orc_cat_norm(self.h)

    def push(self, m, x):
        return lib().orc_cat_push(m.h, self.h, int(x))

    def pop(self, m):
        x = u64(0)
        rc = lib().orc_cat_pop(m.h, self.h, ctypes.byref(x))
        if rc:
            raise RuntimeError(f"oracle pop failed rc={rc}")
        return x.value

    def push_iid(self, m, syms):
        s = np.ascontiguousarray(np.asarray(syms, dtype=np.uint32))
        return lib().orc_iid_push(m.h, self.h, _ptr(s), len(s))

    def pop_iid(self, m, n):
        out = np.zeros(max(n, 1), np.uint32)
        rc = lib().orc_iid_pop(m.h, self.h, _ptr(out), n)
        if rc:
            raise RuntimeError(f"oracle iid pop failed rc={rc}")
        return out[:n]


def uniform_push(m, size, x):
    return lib().orc_uniform_push(m.h, size, x)


def uniform_pop(m, size):
    x = u64(0)
    rc = lib().orc_uniform_pop(m.h, size, ctypes.byref(x))
    if rc:
        raise RuntimeError(f"oracle uniform pop failed rc={rc}")
    return x.value


def encode_chunks(masses, syms, chunk_len, kind=ZEROS, seed=0):
    """Returns (dense stream bytes as np.uint8, offsets u64, lens u64)."""
    masses = np.ascontiguousarray(np.asarray(masses, dtype=np.uint64))
    syms = np.ascontiguousarray(np.asarray(syms, dtype=np.uint32))
    n = len(syms)
    nchunks = (n + chunk_len - 1) // chunk_len
    cap = 6 * n + 16 * nchunks + 16
    out = np.zeros(cap, np.uint8)
    offsets = np.zeros(max(nchunks, 1), np.uint64)
    lens = np.zeros(max(nchunks, 1), np.uint64)
    rc = lib().orc_encode_chunks(_ptr(masses), len(masses), _ptr(syms), n, chunk_len, kind, seed,
                                 _ptr(out), cap, _ptr(offsets), _ptr(lens))
    if rc:
        raise RuntimeError(f"oracle encode failed rc={rc}")
    total = int(lens[:nchunks].sum())
    return out[:total].copy(), offsets[:nchunks].copy(), lens[:nchunks].copy()


def decode_chunks(masses, data, offsets, lens, n, chunk_len, kind=ZEROS, seed=0):
    masses = np.ascontiguousarray(np.asarray(masses, dtype=np.uint64))
    data = np.ascontiguousarray(np.asarray(data, dtype=np.uint8))
    if data.size == 0:
        data = np.zeros(1, np.uint8)
    offsets = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
    lens = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
    out = np.zeros(max(n, 1), np.uint32)
    rc = lib().orc_decode_chunks(_ptr(masses), len(masses), _ptr(data), _ptr(offsets), _ptr(lens), n,
                                 chunk_len, kind, seed, _ptr(out))
    if rc:
        raise RuntimeError(f"oracle decode failed rc={rc}")
    return out[:n]


def gen_iid(masses, seed, start, n):
    masses = np.ascontiguousarray(np.asarray(masses, dtype=np.uint64))
    out = np.zeros(max(n, 1), np.uint32)
    lib().orc_gen_iid(_ptr(masses), len(masses), seed, start, n, _ptr(out))
    return out[:n]


def splitmix64(x):
    return lib().orc_splitmix64(x)


# ---------------------------------------------------------------- graph models (src/graph_codec.rs)
def all_edge_indices(num_nodes, directed, loops):
    """AllEdgeIndices::into_iter (src/graph_codec.rs:187-199), literally: the loops first,
    then `(0..n).flat_map(|j| (0..j).map(|i| (i, j)))`, each followed by (j, i) if directed."""
    out = [(i, i) for i in range(num_nodes)] if loops else []
    for j in range(num_nodes):
        for i in range(j):
            out.append((i, j))
            if directed:
                out.append((j, i))
    return out


def edge_slots(edges, num_nodes, directed, loops):
    """Vectorised position of each edge in all_edge_indices order (-1 outside the alphabet);
    checked against the literal enumeration in tests/test_oracle.py."""
    e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
    i, j = e[:, 0], e[:, 1]
    base = num_nodes if loops else 0
    a, b = np.minimum(i, j), np.maximum(i, j)
    pair = b * (b - 1) // 2 + a
    if directed:
        slot = base + 2 * pair + (i > j)
    else:
        slot = np.where(i < j, base + pair, -1)
    slot = np.where(i == j, i if loops else -1, slot)
    return np.where((i < num_nodes) & (j < num_nodes) & (i >= 0) & (j >= 0), slot, -1)


def dense_set(edges, num_nodes, directed, loops):
    """DenseSetIID::dense (src/graph_codec.rs:133-138) as a u8 indicator vector."""
    n = (num_nodes if loops else 0) + (num_nodes * num_nodes - num_nodes) // (1 if directed else 2)
    s = edge_slots(edges, num_nodes, directed, loops)
    if (s < 0).any():
        raise ValueError("edge outside the alphabet (the reference panics, src/graph_codec.rs:137)")
    d = np.zeros(n, np.uint8)
    d[s] = 1
    return d


# ---- the other static codecs in chunks (the GPU's section 4b): Uniform, LogUniform, Independent
CODEC_UNIFORM, CODEC_LOGUNIFORM, CODEC_INDEPENDENT = 0, 1, 2


def _codec_args(codec, param, tables, tids):
    if codec != CODEC_INDEPENDENT:
        return codec, param, 0, None, None, None, []
    ms = [np.asarray(t, dtype=np.uint64) for t in tables]
    masses = np.ascontiguousarray(np.concatenate(ms))
    nsyms = np.ascontiguousarray(np.array([len(t) for t in ms], np.uint32))
    tids = np.ascontiguousarray(np.asarray(tids, dtype=np.uint32))
    return codec, param, len(ms), _ptr(masses), _ptr(nsyms), _ptr(tids), [masses, nsyms, tids]


def codec_encode_chunks(codec, syms, chunk_len, param=0, tables=None, tids=None, kind=ZEROS, seed=0):
    """Returns (dense bytes, offsets, lens) of IID<Uniform(param)>, IID<LogUniform(param)> or
    Independent<Categorical>(tables, per-position tids), one message per chunk."""
    syms = np.ascontiguousarray(np.asarray(syms, dtype=np.uint64))
    n = len(syms)
    nchunks = (n + chunk_len - 1) // chunk_len
    cap = 16 * n + 16 * nchunks + 16
    out = np.zeros(cap, np.uint8)
    offsets = np.zeros(max(nchunks, 1), np.uint64)
    lens = np.zeros(max(nchunks, 1), np.uint64)
    c, p, nt, mp, np_, tp, keep = _codec_args(codec, param, tables, tids)
    rc = lib().orc_codec_encode_chunks(c, p, nt, mp, np_, tp, _ptr(syms), n, chunk_len, kind, seed, _ptr(out), cap,
                                       _ptr(offsets), _ptr(lens))
    if rc:
        raise RuntimeError(f"oracle codec encode failed rc={rc}")
    total = int(lens[:nchunks].sum())
    return out[:total].copy(), offsets[:nchunks].copy(), lens[:nchunks].copy()


def codec_decode_chunks(codec, data, offsets, lens, n, chunk_len, param=0, tables=None, tids=None, kind=ZEROS, seed=0):
    data = np.ascontiguousarray(np.asarray(data, dtype=np.uint8))
    if data.size == 0:
        data = np.zeros(1, np.uint8)
    offsets = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
    lens = np.ascontiguousarray(np.asarray(lens, dtype=np.uint64))
    out = np.zeros(max(n, 1), np.uint64)
    c, p, nt, mp, np_, tp, keep = _codec_args(codec, param, tables, tids)
    rc = lib().orc_codec_decode_chunks(c, p, nt, mp, np_, tp, _ptr(data), _ptr(offsets), _ptr(lens), n, chunk_len,
                                       kind, seed, _ptr(out))
    if rc:
        raise RuntimeError(f"oracle codec decode failed rc={rc}")
    return out[:n]



# ---- GraphIID (src/graph_codec.rs:19-94) composed literally from the oracle's codecs
def _label_push(m, label, xs):
    """IID<label>::push of xs (src/codec.rs:415-420): ('cat', masses) or ('uniform', size)."""
    kind, p = label
    if kind == "cat":
        return Categorical(p).push_iid(m, xs)
    for x in reversed(list(xs)):
        rc = uniform_push(m, p, int(x))
        if rc:
            return rc
    return 0


def _label_pop(m, label, n):
    kind, p = label
    if kind == "cat":
        return [int(v) for v in Categorical(p).pop_iid(m, n)]
    return [uniform_pop(m, p) for _ in range(n)]


def graph_iid_push(m, num_nodes, node_labels, edges, edge_labels, bern_masses, node, edge, directed, loops):
    """GraphIID::push (src/graph_codec.rs:31-34) on the oracle message m: EdgesIID::push (61-65:
    the labels sorted by the edge index tuple, IID-pushed, then the ErdosRenyi indicator vector),
    then IID<NodeC>::push of the node labels.  node / edge: None (EmptyCodec), ('cat', masses) or
    ('uniform', size).  Returns the first nonzero status."""
    order = sorted(range(len(edges)), key=lambda k: (int(edges[k][0]), int(edges[k][1])))
    if edge is not None:
        rc = _label_push(m, edge, [int(edge_labels[k]) for k in order])
        if rc:
            return rc
    rc = Categorical(bern_masses).push_iid(m, dense_set(np.asarray(edges).reshape(-1, 2), num_nodes, directed, loops))
    if rc:
        return rc
    if node is not None:
        return _label_push(m, node, [int(x) for x in node_labels])
    return 0


def graph_iid_pop(m, num_nodes, bern_masses, node, edge, directed, loops):
    """GraphIID::pop (src/graph_codec.rs:36-38, 67-71): (node labels, edges sorted by (i, j),
    their labels)."""
    nodes = _label_pop(m, node, num_nodes) if node is not None else None
    alpha = all_edge_indices(num_nodes, directed, loops)
    dense = Categorical(bern_masses).pop_iid(m, len(alpha))
    indices = sorted(a for a, b in zip(alpha, dense) if b)
    labels = _label_pop(m, edge, len(indices)) if edge is not None else None
    return nodes, indices, labels
