"""Row f2 probe: DetectFromAudio kernels for rocprofv3 (tools only)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sonido-sonar_amd")]
import sonar
from sonar import shard
ctx = sonar.Context(0)
x = shard.stream_pcm(0, int(600 * 44100)).double().numpy()
for i in range(3):
    t0 = time.perf_counter()
    ct, f = ctx.detect_from_audio(x, 44100)
    print("ms", (time.perf_counter() - t0) * 1e3, ct, flush=True)
