"""FindBestMatches across ranks without a GPU: sonar_merge_matches (host code
of libsonar_gpu.so) on synthetic per-rank top lists, directly and through the torch.distributed
harness (gloo, world 2 and 3), against the single call's order over the concatenated candidates:
similarity descending -- the radix order of its device sort -- with ties in candidate order,
at most MaxCandidates, ranked from 1 (fingerprint/comparison.go:197-263)."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from sonar._abi import Match
from sonar import compare


def _topk(sims, thr, K):
    """The single call on one query's similarity row: (index, similarity) of the kept matches."""
    idx = [i for i in range(len(sims)) if sims[i] >= thr]
    idx.sort(key=lambda i: (-sims[i], i))            # stable: ties keep candidate order
    return idx[:K]


def _local_lists(S, thr, K, lo, hi):
    """Rank-local output of sonar_find_best_matches on candidates [lo, hi) of S (nq x N)."""
    nq = S.shape[0]
    out = (Match * max(1, nq * K))()
    cnt = np.zeros(nq, np.int64)
    for q in range(nq):
        keep = _topk(S[q, lo:hi], thr, K)
        cnt[q] = len(keep)
        for k, c in enumerate(keep):
            m = out[q * K + k]
            m.candidate, m.rank = c, k + 1
            m.similarity.overall_similarity = S[q, lo + c]
            m.similarity.confidence = float(q * 1000 + lo + c)       # identifies the record
    return out, cnt


def _sims(seed, nq, N):
    rng = np.random.default_rng(seed)
    S = np.round(rng.random((nq, N)), 2)                 # many exact ties
    S[:, ::7] = 0.5
    return S


@pytest.mark.parametrize("R,K,thr", [(1, 5, 0.3), (2, 5, 0.3), (3, 4, 0.0), (4, 10, 0.9), (3, 0, 0.1), (5, 64, 0.2)])
def test_merge_equals_single_call(R, K, thr):
    nq, N = 6, 97
    S = _sims(R * 10 + K, nq, N)
    bounds = [N * r // R for r in range(R + 1)]
    lists = [_local_lists(S, thr, K, bounds[r], bounds[r + 1]) for r in range(R)]
    got = compare.merge_matches([l[0] for l in lists], [l[1] for l in lists], bounds[:-1], nq, K)
    for q in range(nq):
        want = _topk(S[q], thr, K)
        assert [m.candidate for m in got[q]] == want
        assert [m.rank for m in got[q]] == list(range(1, len(want) + 1))
        assert [m.similarity.confidence for m in got[q]] == [float(q * 1000 + c) for c in want]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    nq, N, K, thr = 5, 61, 7, 0.25
    S = _sims(42, nq, N)
    lo, hi = N * rank // world, N * (rank + 1) // world
    got = compare.find_best_matches_distributed(_local_lists(S, thr, K, lo, hi), nq, K, hi - lo)
    if rank == world - 1:
        np.save(out_path, np.array([[m.candidate for m in g] + [-1] * (K - len(g)) for g in got]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_merge_gloo(tmp_path, world):
    out = str(tmp_path / "m.npy")
    mp.spawn(_rank_main, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    S = _sims(42, 5, 61)
    for q in range(5):
        want = _topk(S[q], 0.25, 7)
        assert list(got[q][: len(want)]) == want and all(v == -1 for v in got[q][len(want):])


def test_merge_rejects_bad_arguments():
    from sonar._abi import lib
    assert lib().sonar_merge_matches(None, None, None, 2, 3, 4, None, None) != 0
