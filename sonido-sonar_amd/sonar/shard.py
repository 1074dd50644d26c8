"""Frame sharding of one PCM stream across ranks.

Path A is embarrassingly parallel over STFT frames: rank g of G takes frames
[g*F/G, (g+1)*F/G) and needs only the samples those frames touch -- its slice
plus a (W - H)-sample halo into the next shard.  Nothing is exchanged while
computing; afterwards one all-gather (RCCL over xGMI on MI355X, gloo in the CPU
tests) reassembles the feature timeline in frame order.

`stream_pcm` defines the synthetic C2-shaped stream by sample index (the C1
sweep repeated every 10 s plus 0.05 x N(0,1) noise from a counter-based hash),
so every rank generates exactly its own span -- halo included -- on its own
device, and all spans agree with the unsharded stream sample for sample.
"""
from __future__ import annotations

import math

import torch

SR = 44100
# splitmix64 constants as signed 64-bit values
_GOLD = 0x9E3779B97F4A7C15 - (1 << 64)
_MIX1 = 0xBF58476D1CE4E5B9 - (1 << 64)
_MIX2 = 0x94D049BB133111EB - (1 << 64)


def stft_frames(n: int, W: int, H: int) -> int:
    """(n - W) / H + 1 with Go's truncating division (analyzers/spectral.go:409)."""
    return int((n - W) / H) + 1 if n >= W else (1 if n > W - H else 0)


def frame_range(F: int, world: int, rank: int) -> tuple[int, int]:
    """Frames [f0, f1) of `rank`: contiguous, covering [0, F), every boundary inside even, so a
    shard's frame pairs (the headline kernel transforms frames 2p, 2p+1 as one complex FFT) are
    the unsharded run's pairs and the gathered timeline is bit-identical to it (sonar_multi_shard)."""
    def edge(g):
        return F if g >= world else (F * g // world) & ~1
    return edge(rank), edge(rank + 1)


def sample_span(f0: int, f1: int, W: int, H: int) -> tuple[int, int]:
    """Samples [s0, s1) that frames [f0, f1) read: the slice plus its halo."""
    if f1 <= f0:
        return f0 * H, f0 * H
    return f0 * H, (f1 - 1) * H + W


def _splitmix(x: torch.Tensor) -> torch.Tensor:
    """splitmix64 on int64 tensors (wrap-around arithmetic, logical shifts emulated)."""
    def shr(v, k):
        return (v >> k) & ((1 << (64 - k)) - 1)
    x = x + _GOLD
    x = (x ^ shr(x, 30)) * _MIX1
    x = (x ^ shr(x, 27)) * _MIX2
    return x ^ shr(x, 31)


def stream_pcm(s0: int, s1: int, device="cpu", seed: int = 1234, sr: int = SR,
               dtype=torch.float32) -> torch.Tensor:
    """Samples [s0, s1) of the synthetic stream: 0.5 sin(2 pi (100 t + 9900 t^2 / 20)),
    t = (i mod 10 s) / sr, plus 0.05 N(0,1) from Box-Muller over hashed counters."""
    out = torch.empty(max(s1 - s0, 0), dtype=dtype, device=device)
    chunk = 1 << 24
    period = 10 * sr
    for c0 in range(s0, s1, chunk):
        c1 = min(s1, c0 + chunk)
        idx = torch.arange(c0, c1, dtype=torch.int64, device=device)
        t = (idx % period).to(torch.float64) / sr
        v = 0.5 * torch.sin(2 * math.pi * (100.0 * t + 9900.0 * t * t / 20.0))
        h1 = _splitmix(idx * 2 + seed * 0x100000001)
        h2 = _splitmix(idx * 2 + 1 + seed * 0x100000001)
        u1 = ((h1 >> 11) & ((1 << 53) - 1)).to(torch.float64) * (1.0 / (1 << 53))
        u2 = ((h2 >> 11) & ((1 << 53) - 1)).to(torch.float64) * (1.0 / (1 << 53))
        g = torch.sqrt(-2.0 * torch.log1p(-u1)) * torch.cos(2 * math.pi * u2)
        out[c0 - s0:c1 - s0] = (v + 0.05 * g).to(dtype)
    return out


def gather_rows(local: torch.Tensor, world: int, counts: list[int]) -> torch.Tensor:
    """All-gather per-rank row blocks of different lengths (padded to the longest) and
    concatenate them in rank order: the reassembled feature timeline."""
    if world == 1:
        return local
    import torch.distributed as dist
    mx = max(counts)
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)
