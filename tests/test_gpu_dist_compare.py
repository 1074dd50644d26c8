"""FindBestMatches over rank-local galleries on the GPU (comparison.go:197-263,
1107-1152): every rank holds the queries plus its share of the candidates in its own device gallery,
ranks them with sonar_find_best_matches, and the per-rank top MaxCandidates are all-gathered
(torch.distributed gloo here, world 2 and 3 on the box's one device; RCCL on a multi-GPU node) and
merged by sonar_merge_matches.  The merged lists must equal the single-rank call over all candidates
bit for bit (candidate numbering, ranks, match types and every similarity field).  The in-process
multi-device entry (sonar_find_best_matches_multi, one RCCL all-gather) is run on the one device."""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import sonar
from compare_fixtures import gallery
from sonar.compare import Gallery, find_best_matches_distributed, make_cfg

pytestmark = pytest.mark.gpu

N, QUERIES = 64, [0, 5, 17, 63]


def _rec(m):
    return (m.candidate, m.rank, m.match_type, C.string_at(C.addressof(m.similarity), C.sizeof(m.similarity)))


def _single(ctx, thr, K):
    fps = gallery(9, N)
    g = Gallery(ctx)
    g.add(fps)
    res = g.find_best_matches(np.array(QUERIES), None, make_cfg({"similarity_threshold": thr, "max_candidates": K}))
    out = [[_rec(m) for m in r] for r in res]
    g.close()
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, thr, K, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pickle
    ctx = sonar.Context(0)
    fps = gallery(9, N)
    lo, hi = N * rank // world, N * (rank + 1) // world
    g = Gallery(ctx)
    g.add([fps[q] for q in QUERIES] + fps[lo:hi])        # the queries, then this rank's candidates
    Q = len(QUERIES)
    cfg = make_cfg({"similarity_threshold": thr, "max_candidates": K})
    local = g.find_best_matches_raw(np.arange(Q), np.arange(Q, Q + hi - lo), cfg)
    merged = find_best_matches_distributed(local, Q, K, hi - lo)
    if rank == 0:
        with open(out_path, "wb") as f:
            pickle.dump([[_rec(m) for m in r] for r in merged], f)
    g.close()
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("thr,K", [(0.0, 50), (0.5, 3)])
def test_rank_local_galleries_equal_single_rank(ctx, tmp_path, world, thr, K):
    import pickle
    out = str(tmp_path / "merged.pkl")
    mp.spawn(_rank_main, args=(world, _free_port(), thr, K, out), nprocs=world, join=True)
    with open(out, "rb") as f:
        got = pickle.load(f)
    assert got == _single(ctx, thr, K)


def test_find_best_matches_multi_one_device(ctx):
    """sonar_find_best_matches_multi on a one-device sonar_multi (its RCCL all-gather over one rank)."""
    thr, K = 0.2, 6
    m = sonar.Multi([0])
    c0 = m.ctx(0)
    fps = gallery(9, N)
    g = Gallery(c0)
    g.add(fps)
    res = m.find_best_matches([g], [np.array(QUERIES)], None,
                              make_cfg({"similarity_threshold": thr, "max_candidates": K}))
    assert [[_rec(x) for x in r] for r in res] == _single(ctx, thr, K)
    g.close()
    m.close()
