/* demo.c -- a C99 consumer of include/sonar_gpu.h, the way the cgo shim
 * (sonido-sonar_amd/go/sonargpu/sonargpu.go) drives the library: create a context, run path A
 * (sonar_fingerprint: STFT 1024/256 -> mel(40) -> MFCC(13) + descriptors, host buffers) and
 * path B (sonar_dtw), read errors through sonar_last_error, destroy.  Checks what C alone can
 * check (frame counts, finite outputs, a constant-offset DTW path, Go's error text) and prints
 * "demo ok".  Test infrastructure: run by tests/test_gpu_c_abi.py on the GPU box. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sonar_gpu.h"

#define CHECK(cond, ...) do { if (!(cond)) { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); return 1; } } while (0)

int main(void) {
  sonar_ctx* ctx = NULL;
  int rc, i;
  const int64_t n = 3 * 44100;
  double* pcm;
  int64_t F;
  double *mfcc, *rolloff;
  sonar_fp_cfg cfg;
  sonar_fp_out out;
  CHECK(sonar_abi_version() == SONAR_ABI_VERSION, "abi version %d", sonar_abi_version());
  rc = sonar_create(0, &ctx);
  CHECK(rc == SONAR_OK && ctx, "sonar_create: %d", rc);

  pcm = (double*)malloc(sizeof(double) * (size_t)n);
  for (i = 0; i < n; i++) pcm[i] = 0.5 * sin(2.0 * 3.141592653589793 * 440.0 * i / 44100.0);
  F = sonar_stft_frames(n, 1024, 256);
  CHECK(F == (n - 1024) / 256 + 1, "frames %lld", (long long)F);

  sonar_fp_cfg_default(&cfg);
  cfg.window_size = 1024; cfg.hop_size = 256; cfg.sample_rate = 44100;
  cfg.n_filters = 40; cfg.n_mfcc = 13;
  cfg.flags = SONAR_FP_MFCC | SONAR_FP_SPECTRAL;
  cfg.precision = SONAR_F64; cfg.pcm_dtype = SONAR_F64; cfg.out_dtype = SONAR_F64; cfg.device_ptrs = 0;
  memset(&out, 0, sizeof out);
  mfcc = (double*)calloc((size_t)(F * 13), sizeof(double));
  rolloff = (double*)calloc((size_t)F, sizeof(double));
  out.mfcc = mfcc; out.rolloff = rolloff;
  rc = sonar_fingerprint(ctx, pcm, n, &cfg, &out);
  CHECK(rc == SONAR_OK, "sonar_fingerprint: %d %s", rc, sonar_last_error(ctx));
  for (i = 0; i < F * 13; i++) CHECK(isfinite(mfcc[i]), "mfcc[%d] not finite", i);
  /* a 440 Hz tone: 85 % of the energy is reached at the tone's bin (440 * 1024 / 44100 = 10.2) */
  for (i = 0; i < F; i++) CHECK(rolloff[i] > 300.0 && rolloff[i] < 600.0, "rolloff[%d] = %g", i, rolloff[i]);

  /* Go's error text for a signal shorter than one window (analyzers/spectral.go:409-412) */
  rc = sonar_fingerprint(ctx, pcm, 100, &cfg, &out);
  CHECK(rc == SONAR_ERR_TOO_SHORT && strstr(sonar_last_error(ctx), "signal too short"), "short: %d %s", rc,
        sonar_last_error(ctx));

  {
    /* DTW of a sequence against itself delayed by 5 frames: path ends at (N-1, N-1), distance finite */
    enum { N = 300, D = 12, SH = 5 };
    static double q[N * D], r[N * D], pc[2 * N];
    static int32_t pq[2 * N], pr[2 * N];
    double dist = -1;
    int64_t plen = 0;
    int j;
    for (i = 0; i < N; i++)
      for (j = 0; j < D; j++) {
        q[i * D + j] = sin(0.1 * i + j);
        r[i * D + j] = sin(0.1 * (i >= SH ? i - SH : 0) + j);
      }
    rc = sonar_dtw(ctx, q, N, r, N, D, -1, &dist, pq, pr, pc, &plen, NULL, 0);
    CHECK(rc == SONAR_OK, "sonar_dtw: %d %s", rc, sonar_last_error(ctx));
    CHECK(plen >= N && plen <= 2 * N && pq[0] == 0 && pr[0] == 0 && pq[plen - 1] == N - 1 && pr[plen - 1] == N - 1,
          "dtw path len %lld", (long long)plen);
    CHECK(isfinite(dist) && dist >= 0, "dtw distance %g", dist);
    rc = sonar_dtw(ctx, q, 0, r, N, D, -1, &dist, pq, pr, pc, &plen, NULL, 0);
    CHECK(rc == SONAR_ERR_EMPTY && strstr(sonar_last_error(ctx), "empty sequences provided"), "dtw empty: %d", rc);
  }
  sonar_destroy(ctx);
  free(pcm); free(mfcc); free(rolloff);
  printf("demo ok: %lld frames\n", (long long)F);
  return 0;
}
