"""Path B over many stream pairs (BASELINE config C5).

Each pair (query, reference) goes through the reference's alignment pipeline:
MusicFeatureExtractor energy + chroma for both streams
(fingerprint/extractors/music.go:245-259, :327-376, :460-466) and
AlignmentExtractor.ExtractAlignmentFeatures (fingerprint/extractors/alignment.go:139-219):
NCC of the energy envelopes and DTW of the chroma sequences, scored and ranked as in
stats/alignment.go.  Pairs are independent, so N ranks take contiguous pair ranges with no
data-path collective; one all-gather (RCCL over xGMI on MI355X, gloo in the CPU tests)
collects the fixed-size per-pair records afterwards.
"""
from __future__ import annotations

import math

import numpy as np
import torch

SR = 44100
# per-pair record (float64): what a caller of AlignAudioFiles / the C5 bench keeps per pair
RECORD_FIELDS = ["temporal_offset", "offset_confidence", "alignment_similarity", "alignment_quality",
                 "method", "corr_offset_seconds", "dtw_distance", "peak_lag", "lag_seconds_true"]


def pair_range(P: int, world: int, rank: int) -> tuple[int, int]:
    return P * rank // world, P * (rank + 1) // world


def _envelope(n, sr, gen, device, smooth_s=0.5):
    m = int(math.ceil(n / (smooth_s * sr))) + 2
    pts = torch.rand(m, generator=gen, device=device, dtype=torch.float64) * 0.8 + 0.2
    pos = torch.arange(n, device=device, dtype=torch.float64) / (smooth_s * sr)
    i0 = pos.floor().long().clamp_(max=m - 2)
    frac = pos - i0
    return pts[i0] * (1 - frac) + pts[i0 + 1] * frac


def c3_pair_device(seconds: float, lag_s: float, seed: int, env_seed: int, sr: int = SR, device="cuda"):
    """C3's recipe on the device: one-pole (a = 0.95) filtered N(0,1) noise times a 0.5 s
    piecewise-linear random envelope, query = base[lag:lag+n], reference = base[:n].  Returns
    (query, reference) as float64 device tensors.  The one-pole IIR is applied as a 1024-tap
    FIR (0.95^1024 < 1e-22) through an FFT."""
    n = int(round(seconds * sr))
    lag = int(round(lag_s * sr))
    total = n + lag
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    x = torch.randn(total + 1023, generator=gen, device=device, dtype=torch.float64)
    h = 0.95 ** torch.arange(1024, device=device, dtype=torch.float64)
    L = 1 << (x.numel() + 1024).bit_length()
    base = torch.fft.irfft(torch.fft.rfft(x, L) * torch.fft.rfft(h, L), L)[1023:1023 + total]   # causal FIR
    gen.manual_seed(env_seed)
    base = base * _envelope(total, sr, gen, device)
    base = base / base.abs().max()
    return base[lag:lag + n].contiguous(), base[:n].contiguous()


def c5_pair_device(k: int, seconds: float = 60.0, sr: int = SR, device="cuda"):
    """C5 pair k: C3's recipe with seed 1000 + k, envelope seed 5000 + k and a lag uniform in
    [0, 20) s (PCG64 seed 2024 + k).  Returns (query, reference, lag_seconds)."""
    lag_s = float(np.random.Generator(np.random.PCG64(2024 + k)).uniform(0, 20.0))
    q, r = c3_pair_device(seconds, lag_s, 1000 + k, 5000 + k, sr, device)
    return q, r, lag_s


def align_pair(ctx, q, r, sample_rate=SR, stft_window=1024, hop=256, feature_window=1024, max_lag_seconds=60.0,
               lag_seconds_true=float("nan")):
    """Alignment record of one pair; q, r are float64 device tensors (or numpy arrays).  Device
    tensors go through sonar_align_pair_device (features stay in HBM, one C call per pair)."""
    if isinstance(q, torch.Tensor) and isinstance(r, torch.Tensor) and q.is_cuda and r.is_cuda:
        torch.cuda.current_stream(q.device).synchronize()     # q, r were written on torch's stream
        res = ctx.align_pair_device(q.data_ptr(), q.numel(), r.data_ptr(), r.numel(), sample_rate, stft_window, hop,
                                    feature_window, max_lag_seconds)
        return record_of(res, lag_seconds_true), res
    feats = []
    for x in (q, r):
        if isinstance(x, torch.Tensor):
            n = x.numel()
            Fe = (n - feature_window) // hop + 1 if n >= feature_window else 0
            F = (n - stft_window) // hop + 1
            e = torch.empty(max(Fe, 1), dtype=torch.float64, device=x.device)
            c = torch.empty((F, 12), dtype=torch.float64, device=x.device)
            ctx.music_alignment_features_device(x.data_ptr(), n, sample_rate, e.data_ptr(), c.data_ptr(),
                                                stft_window, hop, feature_window, hop)
            torch.cuda.synchronize(x.device)
            feats.append((e[:Fe].cpu().numpy(), c.cpu().numpy(), n))
        else:
            e, c = ctx.music_alignment_features(x, sample_rate, stft_window, hop, feature_window, hop)
            feats.append((e, c, len(x)))
    (qe, qc, nq), (re_, rc, nr) = feats
    res = ctx.align_features(qe, re_, qc, rc, nq, nr, sample_rate, sample_rate, hop, feature_window,
                             max_lag_seconds)
    return record_of(res, lag_seconds_true), res


def record_of(res, lag_seconds_true=float("nan")):
    def g(name, default=float("nan")):
        v = res.get(name)
        return float(np.ravel(v)[0]) if v is not None and np.size(v) else default
    return np.array([g("temporal_offset"), g("offset_confidence"), g("alignment_similarity"),
                     g("alignment_quality"), g("method"), g("corr_offset_seconds"), g("dtw_distance"),
                     g("peak_lag"), lag_seconds_true])


def gather_records(local: torch.Tensor, world: int, counts: list[int]) -> torch.Tensor:
    """All-gather fixed-size per-pair records (rows) from every rank, in pair order."""
    if world == 1:
        return local
    width = local.shape[1]
    cap = max(counts)
    pad = torch.zeros((cap, width), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    torch.distributed.all_gather(parts, pad)
    return torch.cat([p[:c] for p, c in zip(parts, counts)], 0)


def align_pairs(pair_ids, make_pair, sample_rate=SR, max_lag_seconds=20.0, workers=8, device=0, contexts=None):
    """Align many pairs with `workers` concurrent contexts (one HIP stream each).  The per-pair
    kernels (IIR preprocessing, sequential Go-order NCC sums, the DTW band pipeline) are
    latency-bound; independent pairs on separate streams keep the GPU busy.  make_pair(k) ->
    (query, reference, lag_seconds).  Returns the records in pair_ids order."""
    import concurrent.futures as cf
    import threading

    from . import _abi
    local = threading.local()
    made = []

    def ctx_of():
        if not hasattr(local, "ctx"):
            local.ctx = _abi.Context(device)
            made.append(local.ctx)
        return local.ctx

    def one(k):
        ctx = ctx_of()
        q, r, lag = make_pair(k)
        rec, _ = align_pair(ctx, q, r, sample_rate, max_lag_seconds=max_lag_seconds, lag_seconds_true=lag)
        return rec

    with cf.ThreadPoolExecutor(max_workers=workers) as ex:
        recs = list(ex.map(one, pair_ids))
    for c in made:
        c.close()
    return np.array(recs).reshape(len(recs), len(RECORD_FIELDS))
