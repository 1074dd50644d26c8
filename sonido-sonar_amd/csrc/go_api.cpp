// go_api.cpp -- C++ restatement of the Go orchestration above the kernels
// (placeholder; filled in below the first GPU milestone).
#include "../../include/sonar_gpu.h"
#include <cstring>
extern "C" {
void sonar_fingerprint_config_default(sonar_fingerprint_config* c) {
  std::memset(c, 0, sizeof(*c));
  c->window_size = 2048; c->hop_size = 512; c->enable_content_detect = 1; c->window_type = SONAR_WIN_HANN;
}
int sonar_generate_fingerprint(sonar_ctx*, const double*, int64_t, int32_t, const char*, const sonar_fingerprint_config*,
                               sonar_result** out) { if (out) *out = nullptr; return SONAR_ERR_UNSUPPORTED; }
int sonar_align_features(sonar_ctx*, const double*, int64_t, const double*, int64_t, const double*, int64_t,
                         const double*, int64_t, int64_t, int64_t, int32_t, int32_t, int32_t, int32_t, double,
                         sonar_result** out) { if (out) *out = nullptr; return SONAR_ERR_UNSUPPORTED; }
}
