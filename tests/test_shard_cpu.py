"""Multi-rank path A on CPU: frame sharding with halos, per-sample-index synthetic
stream, and the all-gather that reassembles the timeline (gloo, world size 2).
The per-rank compute is the oracle (the device kernel needs a GPU); what is under
test is the sharding arithmetic the multi-GPU bench and product path use."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from sonar import shard

W, H, SR = 1024, 256, 44100


def test_frame_ranges_cover_and_halo():
    for F in (1, 7, 1719, 620153):
        for G in (1, 2, 3, 8):
            rs = [shard.frame_range(F, G, g) for g in range(G)]
            assert rs[0][0] == 0 and rs[-1][1] == F
            assert all(rs[g][1] == rs[g + 1][0] for g in range(G - 1))
            for f0, f1 in rs:
                s0, s1 = shard.sample_span(f0, f1, W, H)
                if f1 > f0:
                    assert shard.stft_frames(s1 - s0, W, H) == f1 - f0     # the span yields exactly its frames


def test_stream_pcm_spans_agree_with_whole():
    full = shard.stream_pcm(0, 50000)
    for s0, s1 in [(0, 1), (123, 4567), (44099, 50000), (30000, 30000)]:
        assert torch.equal(shard.stream_pcm(s0, s1), full[s0:s1])
    x = full.double().numpy()
    assert abs(x.mean()) < 0.02 and 0.3 < x.std() < 0.45                 # sweep (0.354 rms) + 0.05 noise


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, n, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    F = shard.stft_frames(n, W, H)
    f0, f1 = shard.frame_range(F, world, rank)
    s0, s1 = shard.sample_span(f0, f1, W, H)
    pcm = shard.stream_pcm(s0, s1)
    mag = O.stft_mag(pcm.double().numpy(), W, H)
    local = torch.from_numpy(O.mfcc_frames(mag, SR, n_coef=13, n_mels=40))
    counts = [b - a for a, b in (shard.frame_range(F, world, g) for g in range(world))]
    timeline = shard.gather_rows(local, world, counts)
    if rank == 0:
        np.save(out_path, timeline.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_timeline_equals_unsharded(tmp_path, world):
    n = int(2.5 * SR) + 77
    out = str(tmp_path / "timeline.npy")
    mp.spawn(_rank_main, args=(world, _free_port(), n, out), nprocs=world, join=True)
    got = np.load(out)
    pcm = shard.stream_pcm(0, n).double().numpy()
    ref = O.mfcc_frames(O.stft_mag(pcm, W, H), SR, n_coef=13, n_mels=40)
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)
