"""The .history writer (uttt_amd.history) against the reference's own writer, pickle.dump of the
list (self_play_cpp.py:95-99, :125-130): the file loads to an equal list (array bytes, dtypes,
shapes, int values and types) for ragged sizes and every value, and on the reference's golden
self-play games (tests/golden/selfplay.npz). CPU only."""
import pickle

import numpy as np

from conftest import golden


def _ref_list(x, p, v):
    return [[x[i].reshape(9, 9, 3).astype(np.float32), p[i].astype(np.float64), int(v[i])] for i in range(len(x))]


def test_fast_history_equals_pickle_dump():
    from uttt_amd import history as H
    rng = np.random.RandomState(5)
    for n in (0, 1, 2, 3, 17, 1000, 1001, 2503):
        x = (rng.rand(n, 243) < 0.3).astype(np.float32)
        p = rng.dirichlet(np.ones(81), size=n) if n else np.zeros((0, 81))
        v = rng.randint(-1, 2, size=n)
        v[:3] = [-1, 0, 1][:min(n, 3)]
        ref = _ref_list(x, p, v)
        fast = pickle.loads(H.history_bytes(x, p, v))  # bytes made by this test
        assert H.lists_equal(fast, ref)
        assert H.lists_equal(fast, pickle.loads(pickle.dumps(ref)))
        assert all(type(r[2]) is int for r in fast)


def test_fast_history_on_golden_games(tmp_path):
    from uttt_amd import history as H
    d = golden("selfplay.npz")
    n = int(d["lengths"].sum())
    x = d["tensors"][:n].astype(np.float32)
    rec = {"inputs": x.reshape(n, 9, 9, 3), "policies": d["policies"][:n], "values": d["values"][:n].astype(np.int64)}
    path = str(tmp_path / "g.history")
    H.write_history_file([rec], path)
    with open(path, "rb") as fh:
        got = pickle.load(fh)  # written by this test
    ref = _ref_list(x, d["policies"][:n], d["values"][:n])
    assert H.lists_equal(got, ref)
    for i, (xi, pi, vi) in enumerate(got):
        assert np.array_equal(pi.view(np.uint64), d["policies"][i].view(np.uint64)) and vi == int(d["values"][i])


def test_streamed_history_chunks_equal_one_piece(tmp_path, monkeypatch):
    """write_history_file streams ply blocks built from whole games (bounded host memory): with tiny
    blocks, boundaries inside and between games, the file equals the one-piece writer's bytes."""
    from uttt_amd import history as H
    rng = np.random.RandomState(9)
    recs = []
    for g, n in enumerate((1, 5, 2, 9, 1, 1, 13, 4)):
        recs.append({"inputs": (rng.rand(n, 9, 9, 3) < 0.3).astype(np.float32),
                     "policies": rng.dirichlet(np.ones(81), size=n), "values": rng.randint(-1, 2, size=n)})
    x = np.concatenate([r["inputs"].reshape(-1, 243) for r in recs])
    p = np.concatenate([r["policies"] for r in recs])
    v = np.concatenate([r["values"] for r in recs])
    whole = H.history_bytes(x, p, v)
    for cap in (1, 3, 7, 1 << 16):
        monkeypatch.setattr(H, "CHUNK_PLIES", cap)
        path = str(tmp_path / f"c{cap}.history")
        n = H.write_history_file(recs, path)
        with open(path, "rb") as fh:
            got = fh.read()
        assert n == len(got) and got == whole, cap
        assert H.history_bytes(x, p, v) == whole
    path = str(tmp_path / "empty.history")
    H.write_history_file([], path)
    with open(path, "rb") as fh:
        assert pickle.load(fh) == []  # written by this test
