"""CPU: the multi-device entries' shard arithmetic (sonar_multi_shard in the C library, pure
integer code) agrees with the bench harness's sonar/shard.py and pairs.py ranges: shards tile
[0, F), every slice yields exactly its frames, and pair ranges tile [0, P)."""
import sonar
from sonar import pairs, shard

W, H = 1024, 256


def test_multi_shard_matches_harness_and_tiles():
    for n in (1000, 5000, 441000, 2_646_000, 158_760_000):
        F = sonar.stft_frames(n, W, H)
        for G in (1, 2, 3, 8):
            prev = 0
            for g in range(G):
                f0, f1, s0, s1 = sonar.multi_shard(n, W, H, G, g)
                assert (f0, f1) == shard.frame_range(F, G, g)
                assert f0 == prev
                prev = f1
                if f1 > f0:
                    assert 0 <= s0 < s1 <= n
                    assert sonar.stft_frames(s1 - s0, W, H) == f1 - f0
                    if (f1 - 1) * H + W <= n:
                        assert (s0, s1) == shard.sample_span(f0, f1, W, H)
            assert prev == F


def test_pair_ranges_tile():
    for P in (1, 7, 1000):
        for G in (1, 3, 8):
            rs = [pairs.pair_range(P, G, g) for g in range(G)]
            assert rs[0][0] == 0 and rs[-1][1] == P
            assert all(rs[g][1] == rs[g + 1][0] for g in range(G - 1))
