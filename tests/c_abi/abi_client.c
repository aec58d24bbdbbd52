/* A C caller of the handle-level ABI (include/adipose_hip.h), the way a non-Python host would
 * drive the engine: no Python, no torch. Built by adipose_tissue-unet_amd/csrc/Makefile (gcc, C11) next to the
 * library; run by tests/test_abi.py (mode "nogpu": ABI version, error reporting without a device) and
 * tests/test_engine.py (mode "gpu": both presets through adp_create -> adp_set_param -> adp_train_step ->
 * adp_get_grad -> adp_forward -> adp_destroy on device 0, with device buffers from the HIP runtime).
 *
 * usage: abi_client nogpu | gpu     exit status 0 = every check passed; one line per check on stdout. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "../../include/adipose_hip.h"

static int fails = 0;
#define CHECK(cond, ...)                          \
  do {                                            \
    if (cond) {                                   \
      printf("ok   ");                            \
    } else {                                      \
      printf("FAIL ");                            \
      ++fails;                                    \
    }                                             \
    printf(__VA_ARGS__);                          \
    printf("\n");                                 \
  } while (0)

static uint64_t rng = 0x2545F4914F6CDD1Dull;
static float urand(void) {   /* xorshift64*, [0, 1) */
  rng ^= rng >> 12;
  rng ^= rng << 25;
  rng ^= rng >> 27;
  return (float)((rng * 0x2545F4914F6CDD1Dull) >> 40) / (float)(1u << 24);
}

/* Glorot-uniform-like kernels, unit gammas, zero betas / biases / moving means, unit moving variances */
static int init_params(adp_handle* h, int preset) {
  for (int i = 0;; ++i) {
    const char* name = adp_param_name(h, i);
    if (!name) return i;
    const int nslots = preset == ADP_PRESET_UNET_BN && strncmp(name, "dec", 3) == 0 && strstr(name, "_up") ? 2
                       : preset == ADP_PRESET_UNET_BN && strcmp(name, "head") != 0                       ? 5
                                                                                                         : 2;
    for (int slot = 0; slot < nslots; ++slot) {
      size_t n = 0;
      if (adp_param_size(h, name, slot, &n)) return -1;
      float* v = (float*)malloc(n * sizeof(float));
      const int is_gamma = preset == ADP_PRESET_UNET_BN && nslots == 5 && slot == 1;
      const int is_var = preset == ADP_PRESET_UNET_BN && nslots == 5 && slot == 4;
      const float lim = slot == 0 ? sqrtf(6.f / (float)(n / 9 + 64)) : 0.f;
      for (size_t j = 0; j < n; ++j) v[j] = slot == 0 ? (2.f * urand() - 1.f) * lim : (is_gamma || is_var ? 1.f : 0.f);
      const int rc = adp_set_param(h, name, slot, v, n);
      free(v);
      if (rc) return -1;
    }
  }
}

/* one preset: create, parameters, four training steps, one gradient read-back, an eval forward */
static void run_preset(int preset, int dtype, int S, int B) {
  const int C = preset == ADP_PRESET_UNET_BN ? 3 : 1;
  adp_config cfg;
  memset(&cfg, 0, sizeof(cfg));
  cfg.preset = preset;
  cfg.tile = S;
  cfg.max_batch = B;
  cfg.dtype = dtype;
  cfg.deep_supervision = 1;
  cfg.init_nb = 44;
  cfg.levels = 3;
  cfg.base = 16;
  cfg.in_ch = C;
  cfg.dropout_rate = 0.3f;
  cfg.seed = 865;
  adp_handle* h = NULL;
  int rc = adp_create(&cfg, 0, &h);
  CHECK(rc == 0 && h, "preset %d: adp_create (%s)", preset, rc ? adp_last_error() : "");
  if (!h) return;
  const int np = init_params(h, preset);
  CHECK(np > 0, "preset %d: %d parameterised layers set (%s)", preset, np, np > 0 ? "" : adp_last_error());

  const size_t npx = (size_t)B * S * S;
  float* hx = (float*)malloc(npx * C * sizeof(float));
  float* hy = (float*)malloc(npx * sizeof(float));
  for (int b = 0; b < B; ++b)
    for (int yy = 0; yy < S; ++yy)
      for (int xx = 0; xx < S; ++xx) {
        const size_t p = ((size_t)b * S + yy) * S + xx;
        const float dy = yy - S / 2.f - 4.f * b, dx = xx - S / 2.f;
        hy[p] = dy * dy + dx * dx < (S / 4.f) * (S / 4.f) ? 1.f : 0.f;
        for (int c = 0; c < C; ++c) hx[p * C + c] = (hy[p] > 0.f ? 0.8f : -0.8f) + 0.5f * (urand() - 0.5f);
      }
  float *dx_ = NULL, *dy_ = NULL, *dp = NULL;
  hipMalloc((void**)&dx_, npx * C * sizeof(float));
  hipMalloc((void**)&dy_, npx * sizeof(float));
  hipMalloc((void**)&dp, npx * sizeof(float));
  hipMemcpy(dx_, hx, npx * C * sizeof(float), hipMemcpyHostToDevice);
  hipMemcpy(dy_, hy, npx * sizeof(float), hipMemcpyHostToDevice);

  adp_train_cfg tc;
  memset(&tc, 0, sizeof(tc));
  tc.use_hard_mining = preset == ADP_PRESET_ADIPOSE_V3;
  tc.hard_example_ratio = 0.7f;
  tc.epsilon_pos = 0.03f;
  tc.epsilon_neg = 0.07f;
  tc.w_main = 1.f;
  tc.w_aux1 = 0.4f;
  tc.w_aux2 = 0.3f;
  tc.beta1 = 0.9f;
  tc.beta2 = 0.999f;
  tc.eps = 1e-7f;
  tc.weight_decay = 0.01f;
  tc.dropout_rate = -1.f;   /* the handle's build_model dropout */
  float m[6], first = 0.f, last = 0.f;
  int ok = 1;
  for (int step = 0; step < 4; ++step) {
    rc = adp_train_step(h, dx_, dy_, B, &tc, 1e-3f, m, NULL);
    if (rc) { ok = 0; break; }
    for (int i = 0; i < 6; ++i) ok = ok && isfinite(m[i]);
    if (step == 0) first = m[0];
    last = m[0];
  }
  CHECK(ok, "preset %d: four adp_train_step calls, finite metrics (loss %.4f -> %.4f, dice %.4f) %s", preset, first,
        last, m[4], rc ? adp_last_error() : "");
  CHECK(last < first, "preset %d: the loss falls over the steps", preset);

  const char* l0 = adp_param_name(h, 0);
  size_t n0 = 0;
  adp_param_size(h, l0, 0, &n0);
  float* g = (float*)malloc(n0 * sizeof(float));
  rc = adp_get_grad(h, l0, 0, g, n0);
  double gn = 0.0;
  for (size_t j = 0; j < n0; ++j) gn += (double)g[j] * g[j];
  CHECK(rc == 0 && isfinite(gn) && gn > 0.0, "preset %d: adp_get_grad(%s) |g| = %.3e", preset, l0, sqrt(gn));
  free(g);

  rc = adp_forward(h, dx_, B, 0, 0.f, 1.f, 0, dp, NULL);
  hipDeviceSynchronize();
  float* hp = (float*)malloc(npx * sizeof(float));
  hipMemcpy(hp, dp, npx * sizeof(float), hipMemcpyDeviceToHost);
  int in01 = rc == 0;
  double agree = 0.0;
  for (size_t p = 0; p < npx; ++p) {
    in01 = in01 && hp[p] >= 0.f && hp[p] <= 1.f;
    agree += (hp[p] > 0.5f) == (hy[p] > 0.5f);
  }
  CHECK(in01, "preset %d: adp_forward probabilities in [0, 1] (pixel agreement with the labels %.3f) %s", preset,
        agree / (double)npx, rc ? adp_last_error() : "");

  rc = adp_forward(h, dx_, B, 0, 0.f, 1.f, 7, dp, NULL);   /* (n > max_batch is valid: processed in chunks) */
  CHECK(rc != 0 && strstr(adp_last_error(), "tta_mode"), "preset %d: an unknown TTA mode is rejected: %s", preset,
        adp_last_error());
  CHECK(adp_destroy(h) == 0, "preset %d: adp_destroy", preset);
  hipFree(dx_);
  hipFree(dy_);
  hipFree(dp);
  free(hx);
  free(hy);
  free(hp);
}

int main(int argc, char** argv) {
  const int gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
  CHECK(adp_abi_version() == ADP_ABI_VERSION, "adp_abi_version() == %d (header)", ADP_ABI_VERSION);
  adp_config bad;
  memset(&bad, 0, sizeof(bad));
  bad.preset = 7;
  adp_handle* h = NULL;
  const int rc = adp_create(&bad, 0, &h);
  CHECK(rc != 0 && h == NULL && strlen(adp_last_error()) > 0, "adp_create(unknown preset) fails: %s", adp_last_error());
  if (gpu) {
    run_preset(ADP_PRESET_UNET_BN, ADP_DTYPE_BF16, 64, 2);
    run_preset(ADP_PRESET_ADIPOSE_V3, ADP_DTYPE_F32, 64, 2);
  }
  printf("%s: %d failed\n", gpu ? "gpu" : "nogpu", fails);
  return fails ? 1 : 0;
}
