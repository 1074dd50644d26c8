"""The N > 1 path through the HIP library, on the GPU box's one device.

1. bench.py's own multi-rank path: a fresh `torch.distributed.run --nproc-per-node 2` child with
   SONAR_BENCH_ONE_DEVICE=1 (both ranks on device 0) and SONAR_BENCH_BACKEND=gloo (RCCL refuses two
   ranks on one device; the driver's 8-GPU runs use neither override).  The ranks run the sharded
   headline on 2 x 20 s (frame shards with the W-H halo, sonar_fingerprint_device on each rank's
   slice) and a 16-pair C5 slice (pair ranges, sonar_align_pairs), and all-gather the MFCC timeline
   and the pair records.  Asserted: the gathered timeline and records equal the single-process
   product results bit for bit (shard boundaries are even, so the headline kernel's frame pairs are
   the unsharded run's, sonar_multi_shard).
2. The gloo frame-shard harness of tests/test_shard_cpu.py with the product on each rank instead of
   the oracle (world 2 and 3), against the product's unsharded call.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import sonar
from sonar import pairs, shard

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, SR = 1024, 256, 44100


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mfcc_cfg(ctx):
    return ctx.config(window_size=W, hop_size=H, sample_rate=SR, n_filters=40, n_mfcc=13, precision=sonar.F32,
                      pcm_dtype=sonar.F32, out_dtype=sonar.F32, flags=sonar.FP_MFCC)


def test_bench_two_ranks_equal_single_rank(ctx, tmp_path):
    seconds, npairs, c5_seconds = 20.0, 16, 12.0
    env = dict(os.environ, SONAR_BENCH_ONE_DEVICE="1", SONAR_BENCH_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--seconds", str(seconds), "--steps", "2", "--warmup", "1", "--dtw-len", "0",
           "--c5-pairs", str(npairs), "--c5-seconds", str(c5_seconds), "--c5-max-lag", "5", "--c5-workers", "8",
           "--reps", "1", "--no-cpu-baseline", "--no-f64", "--ingest-reps", "0", "--c3-seconds", "0",
           "--c4-seconds", "0", "--c6-gallery", "0", "--c7-seconds", "0", "--hw-queues", "16",
           "--dump-dir", str(tmp_path)]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    line = next(ln for ln in p.stdout.splitlines() if ln.startswith("{"))
    assert '"n_gpus": 2' in line
    timeline = np.load(tmp_path / "mfcc_timeline.npy")
    recs = np.load(tmp_path / "c5_records.npy")

    # single process, the whole 2 x 20 s stream in one call
    n = 2 * int(round(seconds * SR))
    pcm = shard.stream_pcm(0, n, device="cuda")
    F = sonar.stft_frames(n, W, H)
    out = torch.empty((F, 13), dtype=torch.float32, device="cuda")
    ctx.fingerprint_device(pcm.data_ptr(), n, _mfcc_cfg(ctx), mfcc=out.data_ptr())
    torch.cuda.synchronize()
    assert ctx.last_fp_kernel() == "mfcc_pair_kernel"
    assert timeline.shape == (F, 13)
    assert np.array_equal(timeline, out.cpu().numpy())

    data = [pairs.c5_pair_device(k, c5_seconds, device="cuda") for k in range(npairs)]
    torch.cuda.synchronize()
    got = ctx.align_pairs([q.data_ptr() for q, _, _ in data], [r.data_ptr() for _, r, _ in data],
                          nq=[q.numel() for q, _, _ in data], nr=[r.numel() for _, r, _ in data],
                          max_lag_seconds=5.0, workers=8, device_ptrs=True)
    ref = np.stack([got[f] for f in sonar.PAIR_FIELDS] + [np.array([lag for _, _, lag in data])], axis=1)
    assert recs.shape == ref.shape
    assert np.array_equal(np.isnan(recs), np.isnan(ref))
    assert np.array_equal(np.nan_to_num(recs), np.nan_to_num(ref))


def _rank_main(rank, world, port, n, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    F = shard.stft_frames(n, W, H)
    f0, f1 = shard.frame_range(F, world, rank)
    s0, s1 = shard.sample_span(f0, f1, W, H)
    pcm = shard.stream_pcm(s0, s1).numpy()
    c = sonar.Context(0)
    local = torch.from_numpy(c.fingerprint(pcm, _mfcc_cfg(c))["mfcc"]) if f1 > f0 else torch.zeros((0, 13))
    assert c.last_fp_kernel() == "mfcc_pair_kernel" or f1 <= f0
    c.close()
    counts = [b - a for a, b in (shard.frame_range(F, world, g) for g in range(world))]
    timeline = shard.gather_rows(local.float(), world, counts)
    if rank == 0:
        np.save(out_path, timeline.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_frame_shards_with_the_product(ctx, tmp_path, world):
    n = int(2.5 * SR) + 77
    out = str(tmp_path / "timeline.npy")
    mp.get_context("spawn")
    mp.spawn(_rank_main, args=(world, _free_port(), n, out), nprocs=world, join=True)
    got = np.load(out)
    ref = ctx.fingerprint(shard.stream_pcm(0, n).numpy(), _mfcc_cfg(ctx))["mfcc"]
    assert got.shape == ref.shape
    assert np.array_equal(got, ref)
