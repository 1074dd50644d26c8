# C5 throughput split (diagnostics only): pairs/s of the whole pair vs its DTW alone vs its
# features + NCC alone, W host threads each driving its own sonar_ctx (ctypes releases the GIL).
#   python tools/scratch/c5_split.py [pairs] [workers]
import os
import sys
import threading
import time
import ctypes as C

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sonido-sonar_amd"))
import torch  # noqa: E402
from sonar import _abi  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
W = int(sys.argv[2]) if len(sys.argv) > 2 else 16
L = _abi.lib()
sr, n = 44100, 60 * 44100
F = int(L.sonar_stft_frames(n, 1024, 256))
E = int(L.sonar_energy_frames(n, 1024, 256))
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(5)
pcm = [torch.randn(n, generator=g, dtype=torch.float64).to(dev) for _ in range(2)]
chroma = torch.rand(2, F, 12, generator=g, dtype=torch.float64).to(dev)
ctxs = [_abi.Context(0) for _ in range(W)]
cap = 2 * F + 1
bufs = [dict(pq=torch.empty(cap, dtype=torch.int32, device=dev), pr=torch.empty(cap, dtype=torch.int32, device=dev),
             pc=torch.empty(cap, dtype=torch.float64, device=dev), e=torch.empty(2, E, dtype=torch.float64, device=dev),
             c=torch.empty(2, F, 12, dtype=torch.float64, device=dev),
             corr=torch.empty(2 * E + 1, dtype=torch.float64, device=dev)) for _ in range(W)]
torch.cuda.synchronize()


def dtw_only(k):
    b, h = bufs[k], ctxs[k]._h
    dist, P = C.c_double(), C.c_int64()
    rc = L.sonar_dtw(h, C.c_void_p(chroma[0].data_ptr()), F, C.c_void_p(chroma[1].data_ptr()), F, 12, -1,
                     C.byref(dist), C.c_void_p(b["pq"].data_ptr()), C.c_void_p(b["pr"].data_ptr()),
                     C.c_void_p(b["pc"].data_ptr()), C.byref(P), None, 1)
    assert rc == 0, rc


def feats_ncc(k):
    b, x = bufs[k], ctxs[k]
    for s in range(2):
        x.music_alignment_features_device(pcm[s].data_ptr(), n, sr, b["e"][s].data_ptr(), b["c"][s].data_ptr())
    met = (C.c_double * 10)()
    rc = L.sonar_ncc(x._h, C.c_void_p(b["e"][0].data_ptr()), E, C.c_void_p(b["e"][1].data_ptr()), E,
                     int(20 * sr / 256), C.c_void_p(b["corr"].data_ptr()), met, 1)
    assert rc == 0, rc


def full(k):
    ctxs[k].align_pair_device(pcm[0].data_ptr(), n, pcm[1].data_ptr(), n, max_lag_seconds=20.0)


def run(fn, label):
    nxt = [0]
    lock = threading.Lock()

    def worker(k):
        while True:
            with lock:
                i = nxt[0]
                nxt[0] += 1
            if i >= N:
                return
            fn(k)
    for k in range(W):
        fn(k)
    torch.cuda.synchronize()
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(W)]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"{label:12s} W={W:2d}: {N / dt:8.1f} pairs/s  ({dt * 1e3 / N:.3f} ms/pair wall)", flush=True)


which = os.environ.get("C5_SPLIT", "full,dtw,feats")
for name in which.split(","):
    run({"full": full, "dtw": dtw_only, "feats": feats_ncc}[name], name)
