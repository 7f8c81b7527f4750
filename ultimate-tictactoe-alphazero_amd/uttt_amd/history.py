"""The .history file (self_play_cpp.py:95-99, :125-130) written without pickling ply by ply.

The reference's file is ``pickle.dump(history)`` of a flat list of ``[x (9,9,3) f32, policy (81,)
f64, value int]`` plies. Pickling 1.9 M plies (C4: 32,768 games) object by object
takes tens of seconds on one host core, several times the GPUs' self-play time. Every ply after
the first pickles to the same opcode sequence (the numpy reconstructor, ndarray class and dtypes
are memoized by the first ply and referenced by BINGET afterwards), differing only in the array
payloads and the value. So the stream is built from a template taken from the standard pickler
itself: the first ply's bytes verbatim, then one fixed-length record per ply filled in with numpy
(arrays' bytes, value as a 4-byte BININT), one MARK ... APPENDS around all plies, no FRAME opcodes
(optional in protocol 4) and no memo entries for the per-ply objects (nothing refers back to
them). ``pickle.load`` returns a list equal, element by element and type by type, to the one the
reference's writer stores (tests/test_history.py checks that against ``pickle.dumps``).
"""
import pickle
import pickletools
import struct

import numpy as np

_TPL = {}


def _strip(stream, keep_memo_below=None):
    """Opcode stream without FRAME (and, past the first ply, without MEMOIZE) ops: (bytes, [(op, pos)])."""
    ops = [(op.name, pos) for op, _, pos in pickletools.genops(stream)]
    ends = [p for _, p in ops[1:]] + [len(stream)]
    out = bytearray()
    for (name, pos), end in zip(ops, ends):
        if name == "FRAME" or (name == "MEMOIZE" and keep_memo_below is not None and pos >= keep_memo_below):
            continue
        out += stream[pos:end]
    return bytes(out)


def _sentinel(n, dtype, salt):
    """Array whose bytes are unlikely to occur anywhere else in the stream."""
    rng = np.random.RandomState(salt)
    return rng.randint(1 << 20, 1 << 30, size=n).astype(np.float64).astype(dtype) + 0.123


def _template():
    """(head bytes incl. the first ply with marks, later-ply template, offsets of x / policy / value)."""
    if _TPL:
        return _TPL
    x0 = _sentinel(243, np.float32, 1).reshape(9, 9, 3)
    p0 = _sentinel(81, np.float64, 2)
    x1 = _sentinel(243, np.float32, 3).reshape(9, 9, 3)
    p1 = _sentinel(81, np.float64, 4)
    one = pickle.dumps([[x0, p0, 7]], protocol=4)
    two = pickle.dumps([[x0, p0, 7], [x1, p1, 1 << 20]], protocol=4)   # 1 << 20: a BININT ('J') value
    # the second ply's bytes: everything two adds to one between the first ply and the end
    s_two = _strip(two)
    xb1, pb1 = x1.tobytes(), p1.tobytes()
    ix, ip = s_two.find(xb1), s_two.find(pb1)
    iv = s_two.find(b"J" + struct.pack("<i", 1 << 20))
    assert ix > 0 and ip > ix and iv > ip, "unexpected pickle layout"
    # ply 2 starts at its EMPTY_LIST: the op after ply 1's value; find it as the EMPTY_LIST ']' right after
    # the end of the first ply, i.e. at the position where the one-ply stream ends its list item
    s_one = _strip(one)
    # s_one = PROTO EMPTY_LIST MEMOIZE <ply0> APPEND STOP ; s_two = PROTO EMPTY_LIST MEMOIZE MARK <ply0> <ply1> APPENDS STOP
    ply0 = s_one[4:-2]
    assert s_two[4:5] == b"(" and s_two[5:5 + len(ply0)] == ply0, "unexpected pickle layout"
    start = 5 + len(ply0)
    ply1 = s_two[start:-2]
    assert s_two[-2:] == b"e."
    # later plies: drop their MEMOIZE ops (never referenced), keep everything else
    ply1_nomemo = _strip(b"\x80\x04" + ply1 + b".", keep_memo_below=0)[2:-1]
    ox, op_, ov = ply1_nomemo.find(xb1), ply1_nomemo.find(pb1), ply1_nomemo.find(b"J" + struct.pack("<i", 1 << 20))
    assert 0 < ox < op_ < ov
    _TPL.update(head=s_two[:5], ply0=ply0, ply0_x=ply0.find(x0.tobytes()), ply0_p=ply0.find(p0.tobytes()),
                tpl=np.frombuffer(ply1_nomemo, np.uint8), ox=ox, op=op_, ov=ov + 1)
    assert _TPL["ply0_x"] > 0 and _TPL["ply0_p"] > 0
    return _TPL


CHUNK_PLIES = 1 << 16  # plies per body buffer: peak host memory ~ 1.7 KB x this, whatever the file's size


def _ply0(t, x0, p0, v0):
    """The first ply: the standard pickler's bytes (they define the memo entries later plies refer to),
    its payloads replaced and its value re-encoded the way pickle encodes that int."""
    ply0 = bytearray(t["ply0"])
    ply0[t["ply0_x"]:t["ply0_x"] + 972] = x0.tobytes()
    ply0[t["ply0_p"]:t["ply0_p"] + 648] = p0.tobytes()
    vpos = t["ply0_p"] + 648
    tail = bytes(ply0[vpos:])
    # after the payload: BINBYTES trailer ops up to the value opcode 'K\x07' (7 as written above)
    k = tail.rfind(b"K\x07")
    enc = pickle.dumps(int(v0), protocol=4)[2:-1]  # e.g. K\x00 or J\xff\xff\xff\xff (FRAME-free for ints)
    return bytes(ply0[:vpos]) + tail[:k] + enc + tail[k + 2:]


def _body(t, x, policy, value):
    """Later plies (x (m,243) f32, policy (m,81) f64, value (m,) ints) as one uint8 buffer."""
    m = len(x)
    body = np.empty((m, len(t["tpl"])), np.uint8)
    body[:] = t["tpl"]
    body[:, t["ox"]:t["ox"] + 972] = x.view(np.uint8).reshape(m, 972)
    body[:, t["op"]:t["op"] + 648] = policy.view(np.uint8).reshape(m, 648)
    body[:, t["ov"]:t["ov"] + 4] = np.asarray(value).astype("<i4").view(np.uint8).reshape(m, 4)
    return memoryview(body.reshape(-1))


def _norm(x, policy, value):
    return (np.ascontiguousarray(x, dtype=np.float32).reshape(-1, 243),
            np.ascontiguousarray(policy, dtype=np.float64).reshape(-1, 81),
            np.asarray(value, dtype=np.int64).reshape(-1))


def stream_parts(chunks):
    """chunks: an iterable of (x, policy, value) ply blocks, in file order -> the pickle stream of
    their concatenated plies as byte buffers, one body buffer per block (so a caller that feeds
    bounded blocks holds one block's bytes at a time)."""
    t = None
    for x, p, v in chunks:
        x, p, v = _norm(x, p, v)
        if not len(x):
            continue
        if t is None:
            t = _template()
            yield t["head"]
            yield _ply0(t, x[0], p[0], v[0])
            x, p, v = x[1:], p[1:], v[1:]
            if not len(x):
                continue
        yield _body(t, x, p, v)
    if t is None:
        yield pickle.dumps([], protocol=4)
    else:
        yield b"e."


def history_parts(x, policy, value):
    """x (n,9,9,3) f32, policy (n,81) f64, value (n,) ints -> the pickle stream of
    [[x[i], policy[i], int(value[i])] for i in range(n)] as a list of byte buffers."""
    x, policy, value = _norm(x, policy, value)
    return list(stream_parts((x[i:i + CHUNK_PLIES], policy[i:i + CHUNK_PLIES], value[i:i + CHUNK_PLIES])
                             for i in range(0, max(len(x), 1), CHUNK_PLIES)))


def history_bytes(x, policy, value):
    return b"".join(bytes(b) for b in history_parts(x, policy, value))


def _record_chunks(records, cap=None):
    """Per-game records -> ply blocks of about cap plies (whole games), each concatenated on its own."""
    cap = CHUNK_PLIES if cap is None else cap
    buf, n = [], 0
    for r in records:
        buf.append(r)
        n += len(r["values"])
        if n >= cap:
            yield _cat(buf)
            buf, n = [], 0
    if buf:
        yield _cat(buf)


def _cat(recs):
    return (np.concatenate([r["inputs"].reshape(-1, 243) for r in recs]),
            np.concatenate([r["policies"] for r in recs]),
            np.concatenate([r["values"] for r in recs]))


def write_history_file(records, path):
    """records (games sorted by id, each with inputs/policies/values, as SelfPlay.records or the
    gathered records) -> the .history file at path, streamed in blocks of about CHUNK_PLIES plies
    (host memory beyond the records themselves stays ~110 MB at any file size). Returns the byte count."""
    nbytes = 0
    with open(path, "wb") as f:
        for part in stream_parts(_record_chunks(records)):
            f.write(part)
            nbytes += len(part)
    return nbytes


def files_equal(a, b):
    """True when the two .history files load to equal lists (arrays by bytes, dtype and shape)."""
    with open(a, "rb") as fa, open(b, "rb") as fb:
        la, lb = pickle.load(fa), pickle.load(fb)
    return lists_equal(la, lb)


def lists_equal(la, lb):
    if len(la) != len(lb):
        return False
    for ra, rb in zip(la, lb):
        if len(ra) != 3 or len(rb) != 3 or type(ra[2]) is not type(rb[2]) or ra[2] != rb[2]:
            return False
        for u, w in zip(ra[:2], rb[:2]):
            if not (isinstance(u, np.ndarray) and isinstance(w, np.ndarray) and u.dtype == w.dtype
                    and u.shape == w.shape and u.tobytes() == w.tobytes()):
                return False
    return True


__all__ = ["files_equal", "history_bytes", "history_parts", "lists_equal", "stream_parts", "write_history_file"]
