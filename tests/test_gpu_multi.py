"""The batched pair entry (sonar_align_pairs) and the multi-device entries (sonar_multi_*, RCCL)
on the GPU box's one device.  Frames and pairs are independent, so every result must equal the
single-call path exactly:
* sonar_align_pairs records == sonar_align_pair_device per pair (device and host PCM);
* frame sharding: each shard's slice through sonar_fingerprint reproduces its rows of the whole
  (what sonar_fingerprint_multi runs on each device), for G = 3;
* Multi([0]): fingerprint / fingerprint_gather (ncclAllGather) / align_pairs (records through
  ncclAllGather) equal the single-device results."""
import numpy as np
import pytest
import torch

import sonar
from sonar import pairs, synth

pytestmark = pytest.mark.gpu
SR = 44100


def _same(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return a.shape == b.shape and np.array_equal(np.isnan(a), np.isnan(b)) and np.array_equal(
        np.nan_to_num(a), np.nan_to_num(b))


@pytest.fixture(scope="module")
def pair_set():
    ps = [pairs.c5_pair_device(k, 12.0, device="cuda") for k in range(5)]
    torch.cuda.synchronize()
    return ps


def test_align_pairs_equals_per_pair(ctx, pair_set):
    ref = [pairs.align_pair(ctx, q, r, max_lag_seconds=8.0)[0] for q, r, _ in pair_set]
    got = ctx.align_pairs([q.data_ptr() for q, _, _ in pair_set], [r.data_ptr() for _, r, _ in pair_set],
                          nq=[q.numel() for q, _, _ in pair_set], nr=[r.numel() for _, r, _ in pair_set],
                          max_lag_seconds=8.0, workers=3, device_ptrs=True)
    assert np.all(got["status"] == 0)
    for i, f in enumerate(sonar.PAIR_FIELDS):
        assert _same(got[f], [rec[i] for rec in ref]), f
    host = ctx.align_pairs([q.cpu().numpy() for q, _, _ in pair_set], [r.cpu().numpy() for _, r, _ in pair_set],
                           max_lag_seconds=8.0, workers=2)
    for f in sonar.PAIR_FIELDS:
        assert _same(host[f], got[f]), f


def test_align_pairs_reports_bad_pair(ctx):
    """A pair Go rejects ("signal too short ...") fails the call; its record carries the code."""
    q = synth.c3_pair(4.0, 0.5)[0]
    with pytest.raises(sonar.SonarError) as e:
        ctx.align_pairs([q, q[:100]], [q, q], max_lag_seconds=1.0, workers=2)
    assert e.value.code == sonar.ERR_TOO_SHORT if hasattr(sonar, "ERR_TOO_SHORT") else e.value.code == -2


def test_frame_shards_reproduce_whole(ctx):
    x = synth.c2_hour(seconds=30.0)
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=SR, n_filters=40, n_mfcc=13,
                     precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32,
                     flags=sonar.FP_MFCC | sonar.FP_SPECTRAL)
    whole = ctx.fingerprint(x, cfg)
    for g in range(3):
        f0, f1, s0, s1 = sonar.multi_shard(len(x), 1024, 256, 3, g)
        part = ctx.fingerprint(x[s0:s1], cfg)
        for k in ("mfcc", "centroid", "rolloff", "bandwidth", "flatness", "crest", "slope"):
            assert np.array_equal(part[k], whole[k][f0:f1]), (g, k)


@pytest.fixture(scope="module")
def multi():
    m = sonar.Multi([0])
    yield m
    m.close()


def test_multi_fingerprint_equals_single(ctx, multi):
    x = synth.c2_hour(seconds=20.0)
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=SR, n_filters=40, n_mfcc=13,
                     precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32,
                     flags=sonar.FP_MFCC | sonar.FP_MAGNITUDE)
    a = ctx.fingerprint(x, cfg)
    b = multi.fingerprint(x, cfg)
    assert np.array_equal(a["mfcc"], b["mfcc"]) and np.array_equal(a["magnitude"], b["magnitude"])
    cfg.flags = sonar.FP_ZCR
    with pytest.raises(sonar.SonarError):
        multi.fingerprint(x, cfg)


def test_multi_gather_equals_single(ctx, multi):
    x = synth.c2_hour(seconds=20.0)
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=SR, n_filters=40, n_mfcc=13,
                     precision=sonar.F32, pcm_dtype=sonar.F32, out_dtype=sonar.F32, flags=sonar.FP_MFCC)
    ref = ctx.fingerprint(x, cfg)["mfcc"]
    f0, f1, s0, s1 = sonar.multi_shard(len(x), 1024, 256, 1, 0)
    pcm = torch.from_numpy(np.ascontiguousarray(x[s0:s1])).cuda()
    out = torch.full(ref.shape, float("nan"), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    multi.fingerprint_gather([pcm.data_ptr()], len(x), cfg, [out.data_ptr()])
    assert np.array_equal(out.cpu().numpy(), ref)


def test_multi_align_pairs_equals_single(ctx, multi, pair_set):
    qs = [q.cpu().numpy() for q, _, _ in pair_set]
    rs = [r.cpu().numpy() for _, r, _ in pair_set]
    a = ctx.align_pairs(qs, rs, max_lag_seconds=8.0, workers=2)
    b = multi.align_pairs(qs, rs, max_lag_seconds=8.0, workers=2)
    for f in list(sonar.PAIR_FIELDS) + ["status"]:
        assert _same(a[f], b[f]), f


def test_frame_shards_reproduce_whole_f64_pair(ctx):
    """The float64 pair kernel (round 6) under frame sharding: the shards' inner boundaries are even,
    so every shard pairs its frames as the whole does and its rows are the whole's, bit for bit."""
    x = synth.c2_hour(seconds=30.0).astype(np.float64)
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=SR, n_filters=40, n_mfcc=13,
                     precision=sonar.F64, pcm_dtype=sonar.F64, out_dtype=sonar.F64, flags=sonar.FP_MFCC)
    whole = ctx.fingerprint(x, cfg)["mfcc"]
    assert ctx.last_fp_kernel() == "mfcc_pair_kernel"
    for g in range(3):
        f0, f1, s0, s1 = sonar.multi_shard(len(x), 1024, 256, 3, g)
        assert np.array_equal(ctx.fingerprint(x[s0:s1], cfg)["mfcc"], whole[f0:f1]), g


def test_multi_fingerprint_f64_pair_equals_single(ctx, multi):
    x = synth.c2_hour(seconds=20.0).astype(np.float64)
    cfg = ctx.config(window_size=1024, hop_size=256, sample_rate=SR, n_filters=40, n_mfcc=13,
                     precision=sonar.F64, pcm_dtype=sonar.F64, out_dtype=sonar.F64, flags=sonar.FP_MFCC)
    assert np.array_equal(ctx.fingerprint(x, cfg)["mfcc"], multi.fingerprint(x, cfg)["mfcc"])
