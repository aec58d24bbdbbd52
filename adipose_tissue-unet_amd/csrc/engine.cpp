// Handle-level C ABI: native engines for non-Python callers, one per topology preset.
//
//   adp_create(cfg, device, &h)          ADP_PRESET_ADIPOSE_V3: AdiposeUNetV3.build_model (train_adipose_unet_v3.py:
//                                         660-758, segmentation_inference.py:88-146) at tile S;
//                                         ADP_PRESET_UNET_BN: the north-star L-level base-64 BatchNorm U-Net of
//                                         BASELINE.json configs 2/3/5 (nets.UNetBN); buffers for cfg->max_batch
//                                         images x TTA views, allocated once
//   adp_set_param / adp_get_param         Keras layer names and layouts, so a .weights.h5 maps 1:1 (adipose_v3:
//                                         slot 0 kernel, 1 bias; unet_bn: conv 0 kernel, 1 gamma, 2 beta,
//                                         3 moving mean, 4 moving variance; ConvTranspose / head 0 kernel, 1 bias)
//   adp_forward(h, images, n, ...)        predict_single (segmentation_inference.py:153-158) with optional
//                                         TTA (:181-229): z-score + view transform on load, all views of a
//                                         tile batched in one forward, inverse views averaged
//   adp_train_step(h, x, y, n, cfg, lr)   one model.net.fit step (train_adipose_unet_v3.py:1316-1324): forward
//                                         (adipose_v3 with dropout; unet_bn with batch statistics), OHEM /
//                                         BCE+Dice / deep-supervision losses (:217-363, :780-879), backward with
//                                         the bucketed RCCL SUM all-reduce of the gradients on a communication
//                                         stream (each bucket launched as soon as the backward has finished its
//                                         layers, overlapping the remaining backward convs), Adam / AdamW
//   adp_set_comm / adp_comm_*             data parallel over an RCCL communicator (loaded at run time)
//   adp_destroy(h)
//
// The engines are host code over the library's own launchers (adp_conv_fwd, adp_conv_wgrad(_bn), adp_bn_*,
// adp_maxpool2_*, adp_head_*, adp_loss_*, adp_adam, adp_prep_input, adp_tta_merge): the same kernels and
// schedules as nets.AdiposeV3Net / nets.UNetBN with trainer.Trainer / GradBuckets. One handle per device and
// thread; calls are stream-ordered on the caller's stream.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>   // types and enums only: RCCL itself is loaded with dlopen

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "../../include/adipose_hip.h"

namespace adp {
void set_error(const std::string& msg);
int option(const char* name, int dflt);
}

namespace {

int round_up(int x, int m) { return (x + m - 1) / m * m; }

struct DenseL {
  std::string name;
  std::vector<int> cin, cin_s;   // logical / stored input channels per concat part
  int Cin_s = 0, cout = 0, cout_s = 0, dil = 1, up = 0, K = 0, Kpad = 0, Npad = 0, lin = 0, lout = 0;
  std::vector<float> kernel, bias;   // Keras layout (HWIO, [cout])
  void* W = nullptr;                 // packed [Npad][Kpad], compute dtype
  float* b = nullptr;                // [cout_s]
  // training: data-gradient weights [dNpad][dKpad] (adp_pack_weights mode 1), flat-buffer offsets
  void* Wd = nullptr;
  int dNpad = 0, dKpad = 0;
  size_t offW = 0, offB = 0;
};
struct HeadL {
  std::string name;
  int cin = 0, nout = 0, level = 0;
  std::vector<float> kernel, bias;
  float* W = nullptr;   // [nout][cin]
  float* b = nullptr;
  size_t offW = 0, offB = 0;
};

// unet_bn layers (nets.UNetBN.build_layers): kind 0 = 3x3 conv + BatchNorm (no bias), 1 = ConvTranspose 2x2/s2
// (1x1 GEMM over 4*C outputs + pixel-shuffle store, bias), 2 = 1x1 sigmoid head
struct BnLayer {
  std::string name;
  int kind = 0, level = 0;
  std::vector<int> cin, cin_s;   // logical / stored input channels per concat part
  int Cin_s = 0, cout = 0, cout_s = 0, taps = 9, Nout = 0, K = 0, Kpad = 0, Npad = 0, dNpad = 0, dKpad = 0;
  size_t offW = 0, offB = 0, offG = 0, offBeta = 0;   // flat-buffer offsets (nets.ParamStore layout)
  float* st = nullptr;                                // [6][cout_s]: sum, sq, scale, shift, mean, invstd
  float *rmean = nullptr, *rvar = nullptr;            // running statistics (PyTorch semantics)
  void* Wd = nullptr;                                 // data-gradient weights [dNpad][dKpad]
};

#define CK(x)                                              \
  do {                                                     \
    if ((x) != hipSuccess) {                               \
      adp::set_error(std::string("engine: ") + #x);        \
      return -2;                                           \
    }                                                      \
  } while (0)
#define CL(x)                    \
  do {                           \
    const int rc_ = (x);         \
    if (rc_ != 0) return rc_;    \
  } while (0)

// RCCL entry points, resolved once from librccl.so.1 (no link-time dependency: the library loads on
// machines without RCCL, and a process that already holds RCCL gets the same copy back)
struct Rccl {
  bool ok = false;
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommCount) count = nullptr;
  decltype(&ncclAllReduce) allreduce = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
};
Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!lib) lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!lib) return x;
    x.get_id = reinterpret_cast<decltype(x.get_id)>(dlsym(lib, "ncclGetUniqueId"));
    x.init = reinterpret_cast<decltype(x.init)>(dlsym(lib, "ncclCommInitRank"));
    x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(lib, "ncclCommDestroy"));
    x.count = reinterpret_cast<decltype(x.count)>(dlsym(lib, "ncclCommCount"));
    x.allreduce = reinterpret_cast<decltype(x.allreduce)>(dlsym(lib, "ncclAllReduce"));
    x.err = reinterpret_cast<decltype(x.err)>(dlsym(lib, "ncclGetErrorString"));
    x.ok = x.get_id && x.init && x.destroy && x.count && x.allreduce && x.err;
    return x;
  }();
  return r;
}
#define NC(x)                                                                                  \
  do {                                                                                         \
    const ncclResult_t r_ = (x);                                                               \
    if (r_ != ncclSuccess) {                                                                   \
      adp::set_error(std::string("rccl: ") + #x + ": " + (rccl().err ? rccl().err(r_) : "?")); \
      return -3;                                                                               \
    }                                                                                          \
  } while (0)

size_t rup64(size_t x) { return (x + 63) / 64 * 64; }

}  // namespace

struct adp_handle {
  adp_config cfg{};
  int device = 0, es = 4, S = 0, B = 0, nb = 44;
  int cpad[4] = {8, 8, 8, 8}, ch[4] = {0, 0, 0, 0}, sz[4] = {0, 0, 0, 0};
  std::vector<DenseL> dense;
  std::vector<HeadL> heads;
  std::map<std::string, int> dense_idx, head_idx;
  bool dirty = true;
  std::map<std::string, void*> buf;
  float* wstage = nullptr;   // f32 packed staging for the largest layer
  size_t wstage_n = 0;
  // training state (first adp_train_step): one flat f32 buffer each for the master weights P (the
  // dense / head weight and bias pointers point into it), gradients G and Adam moments M, V
  bool train_on = false, host_stale = false, wpack_stale = false;
  float *P = nullptr, *G = nullptr, *Mo = nullptr, *Vo = nullptr;
  size_t nflat = 0, enc_end = 0;
  int step = 0;
  void* comm = nullptr;

  // ---- unet_bn preset (nets.UNetBN): layers, the flat parameter buffers P/G/Mo/Vo (allocated at create),
  // a compute-dtype mirror of P (the forward weights: one cast per step), the per-step statistic arena
  std::vector<BnLayer> bl;
  std::map<std::string, int> bl_idx;
  int levels = 0, base = 64, in_ch = 3;
  void* Pc = nullptr;                 // bf16 mirror of P (forward weights of every layer)
  float *stat_fwd = nullptr, *stat_bwd = nullptr;
  size_t n_stat_fwd = 0, n_stat_bwd = 0;
  std::vector<float*> dtsum;          // per decoder level: [2][Cin_s] channel sums of the concat data gradient
  static constexpr float bn_eps = 1e-5f, bn_momentum = 0.1f;

  // ---- data-parallel gradient buckets (trainer.GradBuckets): reverse flat-buffer order, ~16 MB each; a bucket
  // is SUM-all-reduced on the communication stream as soon as the backward has finished all its layers
  struct Bucket {
    size_t lo = 0, hi = 0;
    std::set<int> layers;
    int pending = 0;
    bool launched = false;
  };
  std::vector<Bucket> buckets;
  std::map<int, int> bucket_of;       // layer id -> bucket
  std::vector<std::pair<size_t, size_t>> layer_span;   // layer id -> [lo, hi) in the flat buffer
  hipStream_t cstream = nullptr;      // RCCL stream
  std::vector<hipEvent_t> bev;        // one "layers done" event per bucket
  hipEvent_t comm_done = nullptr;
  bool dp_active = false;
  float* Gsnap = nullptr;             // adp_debug_grad_flat(which = 1): G as each bucket's all-reduce was issued
  bool deferring = false;             // inside a train step's backward: weight-gradient reductions deferred
  std::string comm_err;

  ~adp_handle() {
    for (auto& l : bl) (void)hipFree(l.Wd);
    if (!bl.empty()) {
      for (auto& l : bl) { (void)hipFree(l.rmean); (void)hipFree(l.rvar); }
      (void)hipFree(Pc);
      (void)hipFree(stat_fwd);
    }
    for (auto e : bev) (void)hipEventDestroy(e);
    if (comm_done) (void)hipEventDestroy(comm_done);
    if (cstream) (void)hipStreamDestroy(cstream);
    if (Gsnap) (void)hipFree(Gsnap);
    for (auto& l : dense) {
      if (!train_on || cfg.dtype != ADP_DTYPE_F32) (void)hipFree(l.W);
      if (!train_on) (void)hipFree(l.b);
      (void)hipFree(l.Wd);
    }
    if (!train_on)
      for (auto& h : heads) { (void)hipFree(h.W); (void)hipFree(h.b); }
    for (auto& kv : buf) (void)hipFree(kv.second);
    (void)hipFree(wstage);
    (void)hipFree(P); (void)hipFree(G); (void)hipFree(Mo); (void)hipFree(Vo);
  }

  int alloc(const char* name, size_t bytes) {
    void* p = nullptr;
    CK(hipMalloc(&p, bytes));
    CK(hipMemset(p, 0, bytes));
    buf[name] = p;
    return 0;
  }
  template <typename T = void>
  T* b(const char* name) { return static_cast<T*>(buf.at(name)); }

  void add_dense(const char* name, int lin, std::vector<int> parts, int lout, int cout, int dil = 1, int up = 0) {
    DenseL l;
    l.name = name;
    l.cin = parts;
    const int in_pad = lin < 0 ? 8 : cpad[lin];
    for (int c : parts) l.cin_s.push_back(round_up(c, in_pad));
    for (int c : l.cin_s) l.Cin_s += c;
    l.cout = cout;
    l.cout_s = round_up(cout, cpad[lout]);
    l.dil = dil;
    l.up = up;
    l.K = 9 * l.Cin_s;
    l.Kpad = round_up(l.K, 32);
    l.Npad = round_up(l.cout_s, 64);
    l.lin = lin;
    l.lout = lout;
    int cin = 0;
    for (int c : parts) cin += c;
    l.kernel.assign((size_t)9 * cin * cout, 0.f);
    l.bias.assign(cout, 0.f);
    dense_idx[name] = (int)dense.size();
    dense.push_back(std::move(l));
  }
  void add_head(const char* name, int cin, int nout, int level) {
    HeadL h;
    h.name = name;
    h.cin = cin;
    h.nout = nout;
    h.level = level;
    h.kernel.assign((size_t)cin * nout, 0.f);
    h.bias.assign(nout, 0.f);
    head_idx[name] = (int)heads.size();
    heads.push_back(std::move(h));
  }

  // Keras HWIO kernel -> packed [Npad][Kpad] (f32 staging) -> compute dtype (nets.Dense.keras_to_packed)
  int upload(hipStream_t s) {
    for (auto& l : dense) {
      std::vector<float> wp((size_t)l.Npad * l.Kpad, 0.f);
      std::vector<int> cm;
      int base = 0;
      for (size_t p = 0; p < l.cin.size(); ++p) {
        for (int c = 0; c < l.cin[p]; ++c) cm.push_back(base + c);
        base += l.cin_s[p];
      }
      const int cin = (int)cm.size();
      for (int t = 0; t < 9; ++t)
        for (int ci = 0; ci < cin; ++ci)
          for (int co = 0; co < l.cout; ++co)
            wp[(size_t)co * l.Kpad + t * l.Cin_s + cm[ci]] = l.kernel[((size_t)t * cin + ci) * l.cout + co];
      std::vector<float> bp(l.cout_s, 0.f);
      std::memcpy(bp.data(), l.bias.data(), sizeof(float) * l.cout);
      CK(hipMemcpy(l.b, bp.data(), sizeof(float) * l.cout_s, hipMemcpyHostToDevice));
      if (cfg.dtype == ADP_DTYPE_F32) {
        CK(hipMemcpy(l.W, wp.data(), sizeof(float) * wp.size(), hipMemcpyHostToDevice));
      } else if (train_on) {   // master copy in P, compute copy packed from it
        CK(hipMemcpy(P + l.offW, wp.data(), sizeof(float) * wp.size(), hipMemcpyHostToDevice));
        CL(adp_pack_weights(cfg.dtype, 0, 9, l.Cin_s, l.cout_s, P + l.offW, l.Kpad, l.W, l.Npad, l.Kpad, s));
      } else {
        CK(hipMemcpy(wstage, wp.data(), sizeof(float) * wp.size(), hipMemcpyHostToDevice));
        CL(adp_pack_weights(cfg.dtype, 0, 9, l.Cin_s, l.cout_s, wstage, l.Kpad, l.W, l.Npad, l.Kpad, s));
        CK(hipStreamSynchronize(s));   // the staging buffer is reused by the next layer
      }
    }
    for (auto& h : heads) {
      std::vector<float> wt((size_t)h.nout * h.cin);
      for (int ci = 0; ci < h.cin; ++ci)
        for (int o = 0; o < h.nout; ++o) wt[(size_t)o * h.cin + ci] = h.kernel[(size_t)ci * h.nout + o];
      CK(hipMemcpy(h.W, wt.data(), sizeof(float) * wt.size(), hipMemcpyHostToDevice));
      CK(hipMemcpy(h.b, h.bias.data(), sizeof(float) * h.nout, hipMemcpyHostToDevice));
    }
    if (train_on) CK(hipStreamSynchronize(s));
    dirty = false;
    wpack_stale = false;
    return 0;
  }

  // P -> host Keras copies (after training steps)
  int download() {
    std::vector<float> wp;
    for (auto& l : dense) {
      wp.resize((size_t)l.Npad * l.Kpad);
      CK(hipMemcpy(wp.data(), P + l.offW, sizeof(float) * wp.size(), hipMemcpyDeviceToHost));
      std::vector<int> cm;
      int base = 0;
      for (size_t p = 0; p < l.cin.size(); ++p) {
        for (int c = 0; c < l.cin[p]; ++c) cm.push_back(base + c);
        base += l.cin_s[p];
      }
      const int cin = (int)cm.size();
      for (int t = 0; t < 9; ++t)
        for (int ci = 0; ci < cin; ++ci)
          for (int co = 0; co < l.cout; ++co)
            l.kernel[((size_t)t * cin + ci) * l.cout + co] = wp[(size_t)co * l.Kpad + t * l.Cin_s + cm[ci]];
      CK(hipMemcpy(l.bias.data(), P + l.offB, sizeof(float) * l.cout, hipMemcpyDeviceToHost));
    }
    for (auto& h : heads) {
      std::vector<float> wt((size_t)h.nout * h.cin);
      CK(hipMemcpy(wt.data(), P + h.offW, sizeof(float) * wt.size(), hipMemcpyDeviceToHost));
      for (int ci = 0; ci < h.cin; ++ci)
        for (int o = 0; o < h.nout; ++o) h.kernel[(size_t)ci * h.nout + o] = wt[(size_t)o * h.cin + ci];
      CK(hipMemcpy(h.bias.data(), P + h.offB, sizeof(float) * h.nout, hipMemcpyDeviceToHost));
    }
    host_stale = false;
    return 0;
  }

  // the last step's gradient of one layer in the Keras layout (slot 0 kernel, 1 bias), from G
  int v3_get_grad(const std::string& name, int slot, float* host) {
    CK(hipDeviceSynchronize());
    auto d = dense_idx.find(name);
    if (d != dense_idx.end()) {
      const DenseL& l = dense[d->second];
      if (slot == 1) {
        CK(hipMemcpy(host, G + l.offB, sizeof(float) * l.cout, hipMemcpyDeviceToHost));
        return 0;
      }
      std::vector<float> wp((size_t)l.Npad * l.Kpad);
      CK(hipMemcpy(wp.data(), G + l.offW, sizeof(float) * wp.size(), hipMemcpyDeviceToHost));
      std::vector<int> cm;
      int base_c = 0;
      for (size_t p = 0; p < l.cin.size(); ++p) {
        for (int c = 0; c < l.cin[p]; ++c) cm.push_back(base_c + c);
        base_c += l.cin_s[p];
      }
      const int cin = (int)cm.size();
      for (int t = 0; t < 9; ++t)
        for (int ci = 0; ci < cin; ++ci)
          for (int co = 0; co < l.cout; ++co)
            host[((size_t)t * cin + ci) * l.cout + co] = wp[(size_t)co * l.Kpad + t * l.Cin_s + cm[ci]];
      return 0;
    }
    const HeadL& h = heads[head_idx.at(name)];
    if (slot == 1) {
      CK(hipMemcpy(host, G + h.offB, sizeof(float) * h.nout, hipMemcpyDeviceToHost));
      return 0;
    }
    std::vector<float> wt((size_t)h.nout * h.cin);
    CK(hipMemcpy(wt.data(), G + h.offW, sizeof(float) * wt.size(), hipMemcpyDeviceToHost));
    for (int ci = 0; ci < h.cin; ++ci)
      for (int o = 0; o < h.nout; ++o) host[(size_t)ci * h.nout + o] = wt[(size_t)o * h.cin + ci];
    return 0;
  }

  // bf16: compute-dtype forward weights from the master copy (every training step, and before an
  // inference forward that follows a step)
  int pack_forward(hipStream_t s) {
    if (cfg.dtype == ADP_DTYPE_F32) return 0;
    for (auto& l : dense)
      CL(adp_pack_weights(cfg.dtype, 0, 9, l.Cin_s, l.cout_s, P + l.offW, l.Kpad, l.W, l.Npad, l.Kpad, s));
    wpack_stale = false;
    return 0;
  }

  int ensure_train() {
    if (train_on) return 0;
    size_t off = 0;
    for (size_t i = 0; i < dense.size(); ++i) {
      auto& l = dense[i];
      l.offW = off;
      off += rup64((size_t)l.Npad * l.Kpad);
      l.offB = off;
      off += rup64(l.cout_s);
      if (l.name == "down3_conv2") enc_end = off;
      l.dNpad = round_up(l.Cin_s, 64) + (l.cin.size() > 1 ? 64 : 0);
      l.dKpad = round_up(9 * l.cout_s, 32);
      CK(hipMalloc(&l.Wd, (size_t)l.dNpad * l.dKpad * es));
      CK(hipMemset(l.Wd, 0, (size_t)l.dNpad * l.dKpad * es));
    }
    for (auto& h : heads) {
      h.offW = off;
      off += rup64((size_t)h.nout * h.cin);
      h.offB = off;
      off += rup64(h.nout);
    }
    nflat = off;
    // layer ids for the gradient buckets: dense layers, then heads; each owns [offW, end of its bias)
    layer_span.clear();
    for (auto& l : dense) layer_span.push_back({l.offW, l.offB + rup64(l.cout_s)});
    for (auto& h : heads) layer_span.push_back({h.offW, h.offB + rup64(h.nout)});
    build_buckets();
    for (float** p : {&P, &G, &Mo, &Vo}) {
      CK(hipMalloc(reinterpret_cast<void**>(p), sizeof(float) * nflat));
      CK(hipMemset(*p, 0, sizeof(float) * nflat));
    }
    for (auto& l : dense) {
      if (cfg.dtype == ADP_DTYPE_F32) {
        (void)hipFree(l.W);
        l.W = P + l.offW;
      }
      (void)hipFree(l.b);
      l.b = P + l.offB;
    }
    for (auto& h : heads) {
      (void)hipFree(h.W);
      (void)hipFree(h.b);
      h.W = P + h.offW;
      h.b = P + h.offB;
    }
    // activations of the training forward and every gradient buffer of nets.AdiposeV3Net.backward
    const size_t B_ = B;
    auto act = [&](const char* n, int lvl, int cidx) { return alloc(n, B_ * sz[lvl] * sz[lvl] * ch[cidx] * es); };
    auto f32 = [&](const char* n, int lvl) { return alloc(n, B_ * sz[lvl] * sz[lvl] * 4); };
    int rc = 0;
    if (cfg.deep_supervision)
      rc = rc || f32("s_aux1", 2) || f32("s_aux2", 1) || f32("p_aux1", 0) || f32("p_aux2", 0) ||
           f32("ds_aux1", 2) || f32("ds_aux2", 1) || act("g_aux_u3", 2, 2) || act("g_aux_u2", 1, 1) ||
           f32("dp_aux1", 0) || f32("dp_aux2", 0);
    rc = rc || f32("dp_main", 0) || act("g_u1", 0, 0);
    for (int lvl = 1; lvl <= 3 && !rc; ++lvl) {
      const int L = lvl - 1;
      const std::string sfx = std::to_string(lvl);
      rc = act(("g_u" + sfx + "b").c_str(), L, L) || act(("g_u" + sfx + "a").c_str(), L, L) ||
           act(("g_skip" + sfx).c_str(), L, L) || act(("g_up" + sfx).c_str(), L, lvl) ||
           act(("g_d" + sfx).c_str(), L, L) || act(("g_d" + sfx + "a").c_str(), L, L);
    }
    rc = rc || act("g_u2", 1, 1) || act("g_u3", 2, 2) || act("g_dsum", 3, 3) || act("g_dz_a", 3, 3) ||
         act("g_dz_b", 3, 3) || act("g_p3", 3, 2) || act("g_p2", 2, 1) || act("g_p1", 1, 0);
    rc = rc || alloc("rows", B_ * S * 3 * 4) || alloc("coef", B_ * S * 3 * 4) || alloc("stats", 3 * 8 * 8) ||
         alloc("lossbuf", 4 * 8);
    if (rc) return rc;
    train_on = true;
    dirty = true;   // re-upload the host copies into P
    return 0;
  }

  int conv(const char* name, int N, const void* srcA, int Hs, const void* srcB, void* out, float* accum,
           hipStream_t s, float drop = 0.f, unsigned seed = 0) {
    const DenseL& l = dense[dense_idx.at(name)];
    adp_conv_desc d{};
    adp_conv_io io{};
    d.N = N;
    d.Hs = Hs;
    d.Ws = Hs;
    d.CA_stride = l.cin_s[0];
    d.CB_stride = l.cin_s.size() > 1 ? l.cin_s[1] : 0;
    d.upsample = l.up;
    d.Ho = d.Wo = Hs * (l.up ? 2 : 1);
    d.stride = 1;
    d.kh = d.kw = 3;
    d.dil = l.dil;
    d.pad = l.dil;
    d.Nout = l.cout_s;
    // real channel counts: the pad weight columns / rows are zeros (adp_conv_desc v19 hints, nets.Dense.real_fwd)
    d.CA_real = l.cin[0];
    d.CB_real = l.cin.size() > 1 ? l.cin[1] : 0;
    d.Nout_real = l.cout;
    d.relu = 1;
    d.out_stride = l.cout_s;
    d.mask_scale = d.mask2_scale = 1.f;
    io.srcA = srcA;
    io.srcB = srcB;
    io.W = l.W;
    io.bias = l.b;
    io.out = out;
    if (accum) {
      d.accum_stride = l.cout_s;
      io.accum = accum;
    }
    d.dropout_rate = drop;
    d.dropout_seed = seed;
    return adp_conv_fwd(cfg.dtype, &d, &io, s);
  }

  const DenseL& D(const char* name) const { return dense[dense_idx.at(name)]; }

  // weight gradient of a dense layer (nets.UNetEngine.wgrad): G[W] (+)= X_tap^T dZ, G[b] (+)= sum dZ
  int wgrad(const char* name, int N, int Hs, const void* srcA, const void* srcB, const void* dZ, hipStream_t s) {
    const DenseL& l = D(name);
    adp_conv_desc d{};
    adp_conv_io io{};
    d.N = N;
    d.Hs = d.Ws = Hs;
    d.CA_stride = l.cin_s[0];
    d.CB_stride = l.cin_s.size() > 1 ? l.cin_s[1] : 0;
    d.upsample = l.up;
    d.Ho = d.Wo = Hs * (l.up ? 2 : 1);
    d.stride = 1;
    d.kh = d.kw = 3;
    d.dil = l.dil;
    d.pad = l.dil;
    d.Nout = l.cout_s;
    d.CA_real = l.cin[0];   // (hints as in conv())
    d.CB_real = l.cin.size() > 1 ? l.cin[1] : 0;
    d.Nout_real = l.cout;
    d.mask_scale = d.mask2_scale = 1.f;
    io.srcA = srcA;
    io.srcB = srcB;
    CL(adp_conv_wgrad(cfg.dtype, &d, &io, dZ, l.cout_s, G + l.offW, G + l.offB, s));
    return ready(dense_id(name), s);
  }

  // data gradient (nets.UNetEngine.dgrad): a forward-shaped launch over dZ with the flipped weights;
  // split: channels < cin_s[0] to out, the rest to out2 (concat inputs); skip_first: only the second part
  int dgrad(const char* name, int N, int H, const void* dZ, void* out, const void* addend, const void* mask,
            float mscale, hipStream_t s, void* out2 = nullptr, const void* mask2 = nullptr, bool split = false,
            bool skip_first = false) {
    const DenseL& l = D(name);
    adp_conv_desc d{};
    adp_conv_io io{};
    d.N = N;
    d.Hs = d.Ws = H;
    d.CA_stride = l.cout_s;
    d.Ho = d.Wo = H;
    d.stride = 1;
    d.kh = d.kw = 3;
    d.dil = l.dil;
    d.pad = l.dil;
    d.Nout = l.Cin_s;
    d.CA_real = l.cout;   // (hints as in conv(): nets.Dense.real_dgrad)
    d.Nout_real = l.cin.size() == 1 ? l.cin[0] : 0;
    d.mask_scale = mscale;
    d.mask2_scale = 1.f;
    io.srcA = dZ;
    io.W = l.Wd;
    int ostride = l.Cin_s;
    if (skip_first) {
      io.W = static_cast<const char*>(l.Wd) + (size_t)l.cin_s[0] * l.dKpad * es;
      d.Nout = l.cin_s[1];
      d.Nout_real = l.cin[1];
      ostride = l.cin_s[1];
      out = out2;
      mask = mask2;
    } else if (split) {
      d.out_mode = 2;
      ostride = l.cin_s[0];
      d.out2_stride = l.cin_s[1];
      d.split_c = l.cin_s[0];
      io.out2 = out2;
      if (mask2) {
        d.mask2_stride = l.cin_s[1];
        io.mask2 = mask2;
      }
    }
    d.out_stride = ostride;
    io.out = out;
    io.addend = addend;
    if (mask) {
      d.mask_stride = ostride;
      io.mask = mask;
    }
    return adp_conv_fwd(cfg.dtype, &d, &io, s);
  }

  // nets.AdiposeV3Net.forward: x (N, S, S, 8) -> main probability map p_main (N, S, S); train: dropout
  // (rate r, seeds sd + 1..4 as the Python schedule) and the deep-supervision heads
  int forward(int N, hipStream_t s, bool train = false, float r = 0.f, unsigned sd = 0) {
    const int dt = cfg.dtype;
    CL(conv("down1_conv1", N, b("x"), sz[0], nullptr, b("d1a"), nullptr, s));
    CL(conv("down1_conv2", N, b("d1a"), sz[0], nullptr, b("d1"), nullptr, s));
    CL(adp_maxpool2_fwd(dt, N, sz[0], sz[0], ch[0], b("d1"), nullptr, nullptr, b("p1"), s));
    CL(conv("down2_conv1", N, b("p1"), sz[1], nullptr, b("d2a"), nullptr, s));
    CL(conv("down2_conv2", N, b("d2a"), sz[1], nullptr, b("d2"), nullptr, s));
    CL(adp_maxpool2_fwd(dt, N, sz[1], sz[1], ch[1], b("d2"), nullptr, nullptr, b("p2"), s));
    CL(conv("down3_conv1", N, b("p2"), sz[2], nullptr, b("d3a"), nullptr, s));
    CL(conv("down3_conv2", N, b("d3a"), sz[2], nullptr, b("d3"), nullptr, s));
    CL(adp_maxpool2_fwd(dt, N, sz[2], sz[2], ch[2], b("d3"), nullptr, nullptr, b("p3"), s));
    // the bottleneck Add: f32 accumulates in the dilated convs' epilogues; bf16 sums the six stored maps
    // in one pass (adp_sum_bf16: the same f32 sum, rounded once; keeps the convs on the persistent kernel)
    const size_t nsum = (size_t)N * sz[3] * sz[3] * ch[3];
    const bool f32 = dt == ADP_DTYPE_F32;
    if (f32) CL(adp_fill_f32(nsum, 0.f, b<float>("dsum_f"), s));
    const char* dl[6] = {"dl1", "dl2", "dl3", "dl4", "dl5", "dl6"};
    const char* dn[6] = {"dilate1", "dilate2", "dilate3", "dilate4", "dilate5", "dilate6"};
    for (int i = 0; i < 6; ++i)
      CL(conv(dn[i], N, i ? b(dl[i - 1]) : b("p3"), sz[3], nullptr, b(dl[i]), f32 ? b<float>("dsum_f") : nullptr, s,
              i == 0 ? r : 0.f, sd + 1));
    void* dsum = f32 ? b("dsum_f") : nullptr;
    if (!f32) {
      const void* maps[6];
      for (int i = 0; i < 6; ++i) maps[i] = b(dl[i]);
      CL(adp_sum_bf16(6, maps, nsum, b("dsum"), s));
      dsum = b("dsum");
    }
    CL(conv("up3_conv1", N, dsum, sz[3], nullptr, b("u3a"), nullptr, s));
    CL(conv("up3_conv2", N, b("d3"), sz[2], b("u3a"), b("u3b"), nullptr, s));
    CL(conv("up3_conv3", N, b("u3b"), sz[2], nullptr, b("u3"), nullptr, s, r, sd + 2));
    CL(conv("up2_conv1", N, b("u3"), sz[2], nullptr, b("u2a"), nullptr, s));
    CL(conv("up2_conv2", N, b("d2"), sz[1], b("u2a"), b("u2b"), nullptr, s));
    CL(conv("up2_conv3", N, b("u2b"), sz[1], nullptr, b("u2"), nullptr, s, r, sd + 3));
    CL(conv("up1_conv1", N, b("u2"), sz[1], nullptr, b("u1a"), nullptr, s));
    CL(conv("up1_conv2", N, b("d1"), sz[0], b("u1a"), b("u1b"), nullptr, s));
    CL(conv("up1_conv3", N, b("u1b"), sz[0], nullptr, b("u1"), nullptr, s, r, sd + 4));
    const HeadL& h = heads[head_idx.at("output_softmax")];
    CL(adp_head_softmax2_fwd(dt, (size_t)N * S * S, ch[0], h.cin, b("u1"), h.W, h.b, nullptr, nullptr,
                             b<float>("p_main"), s));
    if (train && cfg.deep_supervision) {
      const char* src[2] = {"u3", "u2"};
      const char* hn[2] = {"aux_out1", "aux_out2"};
      const char* sb[2] = {"s_aux1", "s_aux2"};
      const char* pb[2] = {"p_aux1", "p_aux2"};
      const int lv[2] = {2, 1};
      for (int k = 0; k < 2; ++k) {
        const HeadL& a = heads[head_idx.at(hn[k])];
        const int z = sz[lv[k]];
        CL(adp_head_sigmoid_fwd(dt, (size_t)N * z * z, ch[lv[k]], a.cin, b(src[k]), a.W, a.b, nullptr, nullptr,
                                b<float>(sb[k]), s));
        CL(adp_resize_bilinear_fwd(N, z, z, S, S, b<float>(sb[k]), b<float>(pb[k]), s));
      }
    }
    return 0;
  }

  // nets.AdiposeV3Net.backward (+ _dec_level): parameter gradients into G from dp_main / dp_aux*
  int backward(int N, float keep, bool full, hipStream_t s) {
    const int dt = cfg.dtype;
    for (auto& l : dense) {
      if (l.name == "down1_conv1") continue;
      const bool enc = l.name.rfind("down", 0) == 0;
      if (!full && (enc || l.name == "dilate1")) continue;
      CL(adp_pack_weights(dt, 1, 9, l.Cin_s, l.cout_s, P + l.offW, l.Kpad, l.Wd, l.dNpad, l.dKpad, s));
    }
    const HeadL& h = heads[head_idx.at("output_softmax")];
    CL(adp_head_softmax2_bwd(dt, (size_t)N * S * S, ch[0], h.cin, b("u1"), h.W, nullptr, nullptr, b<float>("p_main"),
                             b<float>("dp_main"), nullptr, b("u1"), keep, b("g_u1"), G + h.offW, G + h.offB, s));
    CL(ready(head_id("output_softmax"), s));
    const void* aux_add[3] = {nullptr, nullptr, nullptr};   // by level: [1] u2, [2] u3
    if (cfg.deep_supervision) {
      const char* src[2] = {"u3", "u2"};
      const char* hn[2] = {"aux_out1", "aux_out2"};
      const char* sb[2] = {"s_aux1", "s_aux2"};
      const char* dsb[2] = {"ds_aux1", "ds_aux2"};
      const char* dpb[2] = {"dp_aux1", "dp_aux2"};
      const char* dx[2] = {"g_aux_u3", "g_aux_u2"};
      const int lv[2] = {2, 1};
      for (int k = 0; k < 2; ++k) {
        const HeadL& a = heads[head_idx.at(hn[k])];
        const int z = sz[lv[k]];
        CL(adp_resize_bilinear_bwd(N, z, z, S, S, b<float>(dpb[k]), b<float>(dsb[k]), s));
        CL(adp_head_sigmoid_bwd(dt, (size_t)N * z * z, ch[lv[k]], a.cin, b(src[k]), a.W, nullptr, nullptr,
                                b<float>(sb[k]), b<float>(dsb[k]), nullptr, nullptr, 1.f, b(dx[k]), G + a.offW,
                                G + a.offB, s));
        CL(ready(head_id(hn[k]), s));
        aux_add[lv[k]] = b(dx[k]);
      }
    }
    // decoder levels 1 (full resolution), 2, 3
    for (int lvl = 1; lvl <= 3; ++lvl) {
      const int L = lvl - 1;
      const std::string n = std::to_string(lvl);
      const std::string c3 = "up" + n + "_conv3", c2 = "up" + n + "_conv2", c1 = "up" + n + "_conv1";
      void* dz3 = b(("g_u" + n).c_str());
      void* ub = b(("u" + n + "b").c_str());
      void* ua = b(("u" + n + "a").c_str());
      void* gub = b(("g_u" + n + "b").c_str());
      void* gua = b(("g_u" + n + "a").c_str());
      CL(wgrad(c3.c_str(), N, sz[L], ub, nullptr, dz3, s));
      CL(dgrad(c3.c_str(), N, sz[L], dz3, gub, nullptr, ub, 1.f, s));
      CL(wgrad(c2.c_str(), N, sz[L], b(("d" + n).c_str()), ua, gub, s));
      if (full)
        CL(dgrad(c2.c_str(), N, sz[L], gub, b(("g_skip" + n).c_str()), nullptr, nullptr, 1.f, s, gua, ua, true));
      else
        CL(dgrad(c2.c_str(), N, sz[L], gub, nullptr, nullptr, nullptr, 1.f, s, gua, ua, true, true));
      const char* src = lvl == 3 ? (dt == ADP_DTYPE_F32 ? "dsum_f" : "dsum") : (lvl == 2 ? "u3" : "u2");
      CL(wgrad(c1.c_str(), N, sz[lvl], b(src), nullptr, gua, s));
      void* gup = b(("g_up" + n).c_str());
      CL(dgrad(c1.c_str(), N, sz[L], gua, gup, nullptr, nullptr, 1.f, s));
      if (lvl == 3)
        CL(adp_upsample2_bwd(dt, N, sz[3], sz[3], ch[3], gup, nullptr, nullptr, 1.f, b("g_dsum"), s));
      else
        CL(adp_upsample2_bwd(dt, N, sz[lvl], sz[lvl], ch[lvl], gup, aux_add[lvl], b(src), keep,
                             b(lvl == 2 ? "g_u3" : "g_u2"), s));
    }
    // bottleneck: the Add has no activation; dilate_k sees dsum + the chain through dilate_{k+1}
    const size_t nb3 = (size_t)N * sz[3] * sz[3] * ch[3];
    void* gsum = b("g_dsum");
    void* dz = b("g_dz_a");
    void* nz = b("g_dz_b");
    CL(adp_ew_add_mask(dt, nb3, gsum, nullptr, b("dl6"), 1.f, dz, s));
    for (int i = 6; i >= 2; --i) {
      const std::string ln = "dilate" + std::to_string(i), prev = "dl" + std::to_string(i - 1);
      CL(wgrad(ln.c_str(), N, sz[3], b(prev.c_str()), nullptr, dz, s));
      CL(dgrad(ln.c_str(), N, sz[3], dz, nz, gsum, b(prev.c_str()), i == 2 ? keep : 1.f, s));
      std::swap(dz, nz);
    }
    CL(wgrad("dilate1", N, sz[3], b("p3"), nullptr, dz, s));
    if (!full) return 0;
    CL(dgrad("dilate1", N, sz[3], dz, b("g_p3"), nullptr, nullptr, 1.f, s));
    // encoder: pool backward merges the concat-skip gradient and applies the ReLU mask
    for (int lvl = 3; lvl >= 1; --lvl) {
      const int L = lvl - 1;
      const std::string n = std::to_string(lvl);
      void* dd = b(("g_d" + n).c_str());
      void* dz1 = b(("g_d" + n + "a").c_str());
      CL(adp_maxpool2_bwd(dt, N, sz[L], sz[L], ch[L], b(("d" + n).c_str()), nullptr, nullptr,
                          b(("g_p" + n).c_str()), b(("g_skip" + n).c_str()), b(("d" + n).c_str()), 1.f, dd, s));
      const std::string c2 = "down" + n + "_conv2", c1 = "down" + n + "_conv1";
      CL(wgrad(c2.c_str(), N, sz[L], b(("d" + n + "a").c_str()), nullptr, dd, s));
      CL(dgrad(c2.c_str(), N, sz[L], dd, dz1, nullptr, b(("d" + n + "a").c_str()), 1.f, s));
      const char* pin = lvl == 3 ? "p2" : (lvl == 2 ? "p1" : "x");
      CL(wgrad(c1.c_str(), N, sz[L], b(pin), nullptr, dz1, s));
      if (lvl > 1) CL(dgrad(c1.c_str(), N, sz[L], dz1, b(("g_p" + std::to_string(lvl - 1)).c_str()), nullptr, nullptr,
                            1.f, s));
    }
    return 0;
  }

  // ================================================================ data-parallel gradient buckets
  // trainer.GradBuckets: layers in reverse flat-buffer order (the order the backward finishes them), cut into
  // buckets of ~bucket_bytes; a bucket's SUM all-reduce is issued on the communication stream, after an event
  // on the compute stream, as soon as every non-frozen layer of it has reported (ready), so it overlaps the
  // backward launches that follow; dp_finish issues the rest and makes the compute stream wait for all of them
  void build_buckets(size_t bucket_bytes = (size_t)16 << 20) {
    buckets.clear();
    bucket_of.clear();
    std::vector<int> order(layer_span.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return layer_span[a].first > layer_span[b].first; });
    Bucket cur;
    bool open = false;
    for (int id : order) {
      const size_t lo = layer_span[id].first, hi = layer_span[id].second;
      if (open && (cur.hi - lo) * sizeof(float) > bucket_bytes) {
        buckets.push_back(cur);
        open = false;
      }
      if (!open) {
        cur = Bucket();
        cur.hi = hi;
        open = true;
      }
      cur.lo = lo;
      cur.layers.insert(id);
    }
    if (open) buckets.push_back(cur);
    for (size_t b = 0; b < buckets.size(); ++b)
      for (int id : buckets[b].layers) bucket_of[id] = (int)b;
  }
  std::vector<std::set<int>> pend;
  int dp_begin(const std::set<int>& frozen) {
    dp_active = false;
    if (!comm) return 0;
    if (!cstream) {
      CK(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
      CK(hipEventCreateWithFlags(&comm_done, hipEventDisableTiming));
    }
    while (bev.size() < buckets.size()) {
      hipEvent_t e = nullptr;
      CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      bev.push_back(e);
    }
    pend.assign(buckets.size(), {});
    dp_queue.clear();
    for (size_t b = 0; b < buckets.size(); ++b) {
      buckets[b].launched = false;
      for (int id : buckets[b].layers)
        if (!frozen.count(id)) pend[b].insert(id);
    }
    dp_active = true;
    return 0;
  }
  // ready buckets are queued and go out dp_launch_group (option, default 2) at a time behind ONE flush of the deferred
  // weight-gradient reductions (trainer.GradBuckets.launch_group, round 6); dp_finish sends the rest
  std::vector<int> dp_queue;
  int dp_launch_queued(hipStream_t s) {
    if (dp_queue.empty()) return 0;
    if (deferring) {   // the buckets' gradients are final only after the recorded reductions ran
      CL(adp_wgrad_flush(s));
      CL(adp_wgrad_defer(1, s));
    }
    std::vector<int> q;
    q.swap(dp_queue);
    for (int bi : q) CL(dp_launch(bi, s));
    return 0;
  }
  int dp_launch(int bi, hipStream_t s) {
    Bucket& bk = buckets[bi];
    bk.launched = true;
    CK(hipEventRecord(bev[bi], s));
    CK(hipStreamWaitEvent(cstream, bev[bi], 0));
    if (adp::option("dp_snapshot", 0)) {   // test hook: what the all-reduce is about to read
      if (!Gsnap) {
        CK(hipMalloc(reinterpret_cast<void**>(&Gsnap), sizeof(float) * nflat));
        CK(hipMemset(Gsnap, 0, sizeof(float) * nflat));
      }
      CK(hipMemcpyAsync(Gsnap + bk.lo, G + bk.lo, sizeof(float) * (bk.hi - bk.lo), hipMemcpyDeviceToDevice, cstream));
    }
    NC(rccl().allreduce(G + bk.lo, G + bk.lo, bk.hi - bk.lo, ncclFloat32, ncclSum, static_cast<ncclComm_t>(comm),
                        cstream));
    return 0;
  }
  // the layer's parameter gradients are final in stream order on s
  int ready(int id, hipStream_t s) {
    if (!dp_active) return 0;
    auto it = bucket_of.find(id);
    if (it == bucket_of.end()) return 0;
    const int bi = it->second;
    pend[bi].erase(id);
    if (pend[bi].empty() && !buckets[bi].launched &&
        std::find(dp_queue.begin(), dp_queue.end(), bi) == dp_queue.end())
      dp_queue.push_back(bi);
    if ((int)dp_queue.size() >= std::max(1, adp::option("dp_launch_group", 2))) return dp_launch_queued(s);
    return 0;
  }
  // error path between dp_begin and dp_finish: buckets already issued may still read G on the communication
  // stream, so the compute stream waits for them before anything (the next step's zero-fill) writes G again
  void dp_abort(hipStream_t s) {
    if (!dp_active) return;
    dp_active = false;
    dp_queue.clear();
    bool any = false;
    for (auto& b : buckets) any = any || b.launched;
    if (any && hipEventRecord(comm_done, cstream) == hipSuccess) (void)hipStreamWaitEvent(s, comm_done, 0);
  }
  int dp_finish(hipStream_t s) {
    if (!dp_active) return 0;
    for (size_t b = 0; b < buckets.size(); ++b)   // buckets whose layers never reported (frozen only)
      if (!buckets[b].launched && std::find(dp_queue.begin(), dp_queue.end(), (int)b) == dp_queue.end())
        dp_queue.push_back((int)b);
    CL(dp_launch_queued(s));
    CK(hipEventRecord(comm_done, cstream));
    CK(hipStreamWaitEvent(s, comm_done, 0));
    dp_active = false;
    return 0;
  }
  int dense_id(const char* name) const { return dense_idx.at(name); }
  int head_id(const char* name) const { return (int)dense.size() + head_idx.at(name); }

  // ================================================================ unet_bn (nets.UNetBN)
  int ch_of(int lvl) const { return base << lvl; }
  // the input layer's weight gradient computes dz = bn_bwd_apply(dA, z) inside the fused cin8 kernel (bf16, 64
  // outputs: igemm_wgrad_cin8_kernel<true>) and stores none; other shapes need a dz buffer for the apply pass
  bool in_dz_fused() const { return cfg.dtype == ADP_DTYPE_BF16 && base == 64; }
  int side(int lvl) const { return S >> lvl; }
  BnLayer& L(const std::string& n) { return bl[bl_idx.at(n)]; }
  void* wfwd(const BnLayer& l) {   // forward-layout weights in the compute dtype
    return cfg.dtype == ADP_DTYPE_F32 ? static_cast<void*>(P + l.offW)
                                      : static_cast<void*>(static_cast<char*>(Pc) + l.offW * es);
  }
  void add_bl(const std::string& name, int kind, int level, std::vector<int> cin, int cout) {
    BnLayer l;
    l.name = name;
    l.kind = kind;
    l.level = level;
    l.cin = cin;
    for (int c : cin) l.cin_s.push_back(round_up(c, 8));
    for (int c : l.cin_s) l.Cin_s += c;
    l.cout = cout;
    l.cout_s = round_up(cout, 8);
    if (kind == 0) {
      l.taps = 9;
      l.Nout = l.cout_s;
    } else if (kind == 1) {
      l.taps = 1;
      l.Nout = 4 * l.cout_s;
    } else {
      l.taps = 1;
      l.Nout = 1;
    }
    l.K = l.taps * l.Cin_s;
    l.Kpad = round_up(l.K, 32);
    l.Npad = round_up(l.Nout, 64);
    l.dNpad = round_up(l.Cin_s, 64) + (l.cin.size() > 1 ? 64 : 0);
    l.dKpad = round_up((kind == 1 ? 4 : l.taps) * l.cout_s, 32);
    bl_idx[name] = (int)bl.size();
    bl.push_back(std::move(l));
  }

  int create_unet_bn() {
    const int Lv = levels;
    int cin = in_ch;
    for (int i = 0; i < Lv; ++i) {
      add_bl("enc" + std::to_string(i) + "_conv1", 0, i, {cin}, ch_of(i));
      add_bl("enc" + std::to_string(i) + "_conv2", 0, i, {ch_of(i)}, ch_of(i));
      cin = ch_of(i);
    }
    for (int i = Lv - 2; i >= 0; --i) {
      const std::string n = "dec" + std::to_string(i);
      add_bl(n + "_up", 1, i, {ch_of(i + 1)}, ch_of(i));
      add_bl(n + "_conv1", 0, i, {ch_of(i), ch_of(i)}, ch_of(i));
      add_bl(n + "_conv2", 0, i, {ch_of(i)}, ch_of(i));
    }
    add_bl("head", 2, 0, {ch_of(0)}, 1);
    // flat layout of nets.ParamStore (W, [b], [gamma, beta] per layer, 64-float aligned slices)
    size_t off = 0;
    for (auto& l : bl) {
      const size_t lo = off;
      l.offW = off;
      off += rup64(l.kind == 2 ? (size_t)l.cin[0] : (size_t)l.Npad * l.Kpad);
      if (l.kind == 0) {
        l.offG = off;
        off += rup64(l.cout_s);
        l.offBeta = off;
        off += rup64(l.cout_s);
      } else {
        l.offB = off;
        off += rup64(l.kind == 2 ? 1 : l.cout_s);
      }
      layer_span.push_back({lo, off});
    }
    nflat = off;
    for (float** p : {&P, &G, &Mo, &Vo}) {
      CK(hipMalloc(reinterpret_cast<void**>(p), sizeof(float) * nflat));
      CK(hipMemset(*p, 0, sizeof(float) * nflat));
    }
    if (cfg.dtype != ADP_DTYPE_F32) {
      CK(hipMalloc(&Pc, (size_t)es * nflat));
      CK(hipMemset(Pc, 0, (size_t)es * nflat));
    }
    n_stat_fwd = 0;
    n_stat_bwd = 0;
    for (auto& l : bl) {
      if (l.kind == 0) n_stat_fwd += 6 * (size_t)l.cout_s;
      if (l.kind == 0 && l.cin.size() > 1) n_stat_bwd += 2 * (size_t)l.Cin_s;
    }
    CK(hipMalloc(reinterpret_cast<void**>(&stat_fwd), sizeof(float) * (n_stat_fwd + n_stat_bwd)));
    CK(hipMemset(stat_fwd, 0, sizeof(float) * (n_stat_fwd + n_stat_bwd)));
    stat_bwd = stat_fwd + n_stat_fwd;
    size_t so = 0, sb = 0;
    dtsum.assign(Lv > 1 ? Lv - 1 : 0, nullptr);
    for (auto& l : bl) {
      if (l.kind == 0) {
        l.st = stat_fwd + so;
        so += 6 * (size_t)l.cout_s;
        CK(hipMalloc(reinterpret_cast<void**>(&l.rmean), sizeof(float) * l.cout_s));
        CK(hipMalloc(reinterpret_cast<void**>(&l.rvar), sizeof(float) * l.cout_s));
        CK(hipMemset(l.rmean, 0, sizeof(float) * l.cout_s));
        CL(adp_fill_f32(l.cout_s, 1.f, l.rvar, nullptr));
        CL(adp_fill_f32(l.cout_s, 1.f, P + l.offG, nullptr));   // Keras / torch BatchNorm init: gamma 1
        if (l.cin.size() > 1) {
          dtsum[l.level] = stat_bwd + sb;
          sb += 2 * (size_t)l.Cin_s;
        }
      }
      if (l.name != "enc0_conv1" && l.kind != 2) {
        CK(hipMalloc(&l.Wd, (size_t)l.dNpad * l.dKpad * es));
        CK(hipMemset(l.Wd, 0, (size_t)l.dNpad * l.dKpad * es));
      }
    }
    CK(hipDeviceSynchronize());
    // activations (nets.UNetBN.alloc) and the gradient buffers of its backward, for max_batch images
    const size_t B_ = B;
    auto act = [&](const std::string& n, int lvl) {
      return alloc(n.c_str(), B_ * side(lvl) * side(lvl) * ch_of(lvl) * es);
    };
    int rc = alloc("x", B_ * S * S * 8 * es);
    for (int i = 0; i < Lv && !rc; ++i) {
      const std::string k = std::to_string(i);
      rc = act("z" + k + "_1", i) || act("z" + k + "_2", i) || act("az" + k + "_1", i) || act("az" + k + "_2", i) ||
           act("dA_z" + k + "_2", i) || act("dz_z" + k + "_2", i) || act("dA_z" + k + "_1", i) ||
           ((i == 0 && in_dz_fused()) ? 0 : act("dz_z" + k + "_1", i));
      if (!rc && i < Lv - 1)
        rc = act("y" + k + "_1", i) || act("y" + k + "_2", i) || act("ay" + k + "_1", i) || act("ay" + k + "_2", i) ||
             act("t" + k, i) || act("dz_y" + k + "_2", i) || act("dA_y" + k + "_1", i) ||
             act("dz_y" + k + "_1", i) || act("skip" + k, i) || act("dt" + k, i) || act("dA_up" + k, i + 1) ||
             alloc(("pool" + k).c_str(), B_ * side(i + 1) * side(i + 1) * ch_of(i) * es) ||
             alloc(("dpool" + k).c_str(), B_ * side(i + 1) * side(i + 1) * ch_of(i) * es);
    }
    if (rc) return rc;
    size_t wmax = 0;   // eval: one layer's forward weights with its BatchNorm scale folded in (bn_conv)
    for (auto& l : bl)
      if (l.kind == 0) wmax = std::max(wmax, (size_t)l.Npad * l.Kpad);
    rc = alloc("wfold", wmax * es);
    if (rc) return rc;
    rc = alloc("p", B_ * S * S * 4) || alloc("dp_main", B_ * S * S * 4) || alloc("probs", B_ * S * S * 4) ||
         alloc("rows", B_ * S * 3 * 4) || alloc("coef", B_ * S * 3 * 4) || alloc("stats", 3 * 8 * 8) ||
         alloc("lossbuf", 4 * 8);
    if (rc) return rc;
    build_buckets();
    train_on = true;
    dirty = false;
    return 0;
  }

  // -- launch helpers (the descriptors ops.conv_fwd / ops.conv_wgrad build for nets.UNetBN)
  static adp_conv_desc desc3(int N, int H, const BnLayer& l) {
    adp_conv_desc d{};
    d.N = N;
    d.Hs = d.Ws = H;
    d.CA_stride = l.cin_s[0];
    d.CB_stride = l.cin_s.size() > 1 ? l.cin_s[1] : 0;
    d.Ho = d.Wo = H;
    d.stride = 1;
    d.kh = d.kw = 3;
    d.dil = 1;
    d.pad = 1;
    d.Nout = l.cout_s;
    d.out_stride = l.cout_s;
    d.mask_scale = d.mask2_scale = 1.f;
    return d;
  }
  float* stv(const BnLayer& l, int k) const { return l.st + (size_t)k * l.cout_s; }
  // conv -> BatchNorm statistics (epilogue, folded by the finalize) -> scale / shift -> relu(bn) materialised
  // (with its 2x2 max-pool when pool != nullptr; act == nullptr: the consumer applies it on load)
  // bnA (training): srcA is layer bnA's pre-BatchNorm output, applied on load; its activation is stored to act_in by
  // this launch (adp_conv_io.act_outA; nets.UNetBN.fuse_bn_load)
  int bn_conv(const std::string& name, int N, const void* srcA, const void* srcB, void* out, void* act, void* pool,
              bool train, hipStream_t s, const BnLayer* bnA = nullptr, void* act_in = nullptr) {
    BnLayer& l = L(name);
    const int H = side(l.level), C = l.cout_s;
    adp_conv_desc d = desc3(N, H, l);
    adp_conv_io io{};
    io.srcA = srcA;
    io.srcB = srcB;
    io.W = wfwd(l);
    io.out = out;
    if (bnA) {
      io.bn_scaleA = stv(*bnA, 2);
      io.bn_shiftA = stv(*bnA, 3);
      io.act_outA = act_in;
    }
    if (!train && act) {
      // eval (nets.UNetBN._conv_eval_folded): the running-statistics BatchNorm is affine, so its scale goes into
      // the weights (f32 master rows x scale -> compute dtype) and its shift + ReLU into the conv epilogue, which
      // writes relu(bn(z)) straight into act: no z round trip, no separate apply pass
      CL(adp_bn_finalize(C, -1.f, l.rmean, l.rvar, P + l.offG, P + l.offBeta, bn_eps, 0.f, stv(l, 2), stv(l, 3),
                         stv(l, 4), stv(l, 5), nullptr, nullptr, s));
      void* wf = b("wfold");
      CL(adp_scale_rows(cfg.dtype, l.Npad, l.Kpad, P + l.offW, l.Kpad, stv(l, 2), C, wf, l.Kpad, s));
      io.W = wf;
      io.bias = stv(l, 3);
      io.out = act;
      d.relu = 1;
      CL(adp_conv_fwd(cfg.dtype, &d, &io, s));
      if (pool) CL(adp_maxpool2_fwd(cfg.dtype, N, H, H, C, act, nullptr, nullptr, pool, s));
      return 0;
    }
    if (train) {
      io.bn_sum = stv(l, 0);
      io.bn_sqsum = stv(l, 1);
      d.bn_defer_fold = 1;
    }
    CL(adp_conv_fwd(cfg.dtype, &d, &io, s));
    if (train)
      CL(adp_bn_finalize_fold(C, (float)((double)N * H * H), stv(l, 0), stv(l, 1), P + l.offG, P + l.offBeta, bn_eps,
                              bn_momentum, stv(l, 2), stv(l, 3), stv(l, 4), stv(l, 5), l.rmean, l.rvar, s));
    else   // eval: (count < 0) the running statistics stand in for the batch sums
      CL(adp_bn_finalize(C, -1.f, l.rmean, l.rvar, P + l.offG, P + l.offBeta, bn_eps, 0.f, stv(l, 2), stv(l, 3),
                         stv(l, 4), stv(l, 5), nullptr, nullptr, s));
    if (pool) CL(adp_bn_apply_maxpool2(cfg.dtype, N, H, H, C, out, stv(l, 2), stv(l, 3), act, pool, s));
    else if (act) CL(adp_bn_apply(cfg.dtype, (size_t)N * H * H, C, out, stv(l, 2), stv(l, 3), act, s));
    return 0;
  }
  int convt_fwd(const std::string& name, int N, const void* src, void* out, hipStream_t s) {
    BnLayer& l = L(name);
    adp_conv_desc d{};
    d.N = N;
    d.Hs = d.Ws = d.Ho = d.Wo = side(l.level + 1);
    d.CA_stride = l.cin_s[0];
    d.stride = 1;
    d.kh = d.kw = 1;
    d.dil = 1;
    d.pad = 0;
    d.Nout = l.Nout;
    d.out_stride = l.cout_s;
    d.out_mode = 1;
    d.shuffle_c = l.cout_s;
    d.mask_scale = d.mask2_scale = 1.f;
    adp_conv_io io{};
    io.srcA = src;
    io.W = wfwd(l);
    io.bias = P + l.offB;
    io.out = out;
    return adp_conv_fwd(cfg.dtype, &d, &io, s);
  }
  int bn_forward(int N, bool train, hipStream_t s) {
    if (cfg.dtype != ADP_DTYPE_F32) CL(adp_cast(ADP_DTYPE_F32, cfg.dtype, nflat, P, Pc, s));
    if (train) CL(adp_fill_f32(n_stat_fwd, 0.f, stat_fwd, s));
    const int Lv = levels;
    const void* src = b("x");
    // training, bf16, 64-channel levels: conv2 applies conv1's BatchNorm-ReLU on load and stores the activation
    // (nets.UNetBN.fuse_bn_load)
    auto bnl = [&](int i) { return train && cfg.dtype == ADP_DTYPE_BF16 && L("enc" + std::to_string(i) + "_conv1").cout_s == 64; };
    for (int i = 0; i < Lv; ++i) {
      const std::string k = std::to_string(i);
      const bool f = bnl(i);
      CL(bn_conv("enc" + k + "_conv1", N, src, nullptr, b(("z" + k + "_1").c_str()),
                 f ? nullptr : b(("az" + k + "_1").c_str()), nullptr, train, s));
      CL(bn_conv("enc" + k + "_conv2", N, b((f ? "z" + k + "_1" : "az" + k + "_1").c_str()), nullptr,
                 b(("z" + k + "_2").c_str()), b(("az" + k + "_2").c_str()), i < Lv - 1 ? b(("pool" + k).c_str()) : nullptr,
                 train, s, f ? &L("enc" + k + "_conv1") : nullptr, f ? b(("az" + k + "_1").c_str()) : nullptr));
      if (i < Lv - 1) src = b(("pool" + k).c_str());
    }
    const void* prev = b(("az" + std::to_string(Lv - 1) + "_2").c_str());
    for (int i = Lv - 2; i >= 0; --i) {
      const std::string k = std::to_string(i);
      CL(convt_fwd("dec" + k + "_up", N, prev, b(("t" + k).c_str()), s));
      const bool f = bnl(i);
      CL(bn_conv("dec" + k + "_conv1", N, b(("az" + k + "_2").c_str()), b(("t" + k).c_str()),
                 b(("y" + k + "_1").c_str()), f ? nullptr : b(("ay" + k + "_1").c_str()), nullptr, train, s));
      // level 0 in training: relu(bn(y0_2)) is only read by the head, which applies it on load; in eval the
      // folded conv writes it (nets.UNetBN.forward: head_bn only when training)
      CL(bn_conv("dec" + k + "_conv2", N, b((f ? "y" + k + "_1" : "ay" + k + "_1").c_str()), nullptr,
                 b(("y" + k + "_2").c_str()), i == 0 && train ? nullptr : b(("ay" + k + "_2").c_str()), nullptr, train, s,
                 f ? &L("dec" + k + "_conv1") : nullptr, f ? b(("ay" + k + "_1").c_str()) : nullptr));
      prev = b(("ay" + k + "_2").c_str());
    }
    const BnLayer& h = L("head");
    const BnLayer& l0 = L("dec0_conv2");
    if (train)
      CL(adp_head_sigmoid_fwd(cfg.dtype, (size_t)N * S * S, l0.cout_s, h.cin[0], b("y0_2"), P + h.offW, P + h.offB,
                              stv(l0, 2), stv(l0, 3), b<float>("p"), s));
    else
      CL(adp_head_sigmoid_fwd(cfg.dtype, (size_t)N * S * S, l0.cout_s, h.cin[0], b("ay0_2"), P + h.offW, P + h.offB,
                              nullptr, nullptr, b<float>("p"), s));
    return 0;
  }

  // -- backward launches
  int bn_dgrad(const std::string& name, int N, const void* dZ, void* out, const std::string& red, const void* redz,
               hipStream_t s) {
    BnLayer& l = L(name);
    const int H = side(l.level);
    adp_conv_desc d = desc3(N, H, l);
    d.CA_stride = l.cout_s;
    d.CB_stride = 0;
    d.Nout = l.Cin_s;
    d.out_stride = l.Cin_s;
    adp_conv_io io{};
    io.srcA = dZ;
    io.W = l.Wd;
    io.out = out;
    if (!red.empty()) {   // the BatchNorm-backward reduction of the layer `out` is the gradient of
      BnLayer& r = L(red);
      d.bnr_stride = r.cout_s;
      io.bnr_z = redz;
      io.bnr_scale = stv(r, 2);
      io.bnr_shift = stv(r, 3);
      io.bnr_mean = stv(r, 4);
      io.bnr_invstd = stv(r, 5);
      io.bnr_dgamma = G + r.offG;
      io.bnr_dbeta = G + r.offBeta;
    }
    return adp_conv_fwd(cfg.dtype, &d, &io, s);
  }
  int convt_dgrad(const std::string& name, int N, const void* dZ, void* out, const std::string& red, const void* redz,
                  hipStream_t s) {
    BnLayer& l = L(name);
    const int H = side(l.level + 1);
    adp_conv_desc d{};
    d.N = N;
    d.Hs = d.Ws = 2 * H;
    d.CA_stride = l.cout_s;
    d.Ho = d.Wo = H;
    d.stride = 2;
    d.kh = d.kw = 2;
    d.dil = 1;
    d.pad = 0;
    d.Nout = l.Cin_s;
    d.out_stride = l.Cin_s;
    d.mask_scale = d.mask2_scale = 1.f;
    adp_conv_io io{};
    io.srcA = dZ;
    io.W = l.Wd;
    io.out = out;
    BnLayer& r = L(red);
    d.bnr_stride = r.cout_s;
    io.bnr_z = redz;
    io.bnr_scale = stv(r, 2);
    io.bnr_shift = stv(r, 3);
    io.bnr_mean = stv(r, 4);
    io.bnr_invstd = stv(r, 5);
    io.bnr_dgamma = G + r.offG;
    io.bnr_dbeta = G + r.offBeta;
    return adp_conv_fwd(cfg.dtype, &d, &io, s);
  }
  // weight gradient of a BatchNorm conv over dz = bn_bwd_apply(dA, z) (computed inside the launch where the halo
  // kernel takes the shape, adp_conv_wgrad_bn); dA == nullptr: dz is already stored
  int bn_wgrad(const std::string& name, int N, const void* srcA, const void* srcB, const void* dA, const void* z,
               void* dz, hipStream_t s) {
    BnLayer& l = L(name);
    const int H = side(l.level);
    adp_conv_desc d = desc3(N, H, l);
    adp_conv_io io{};
    io.srcA = srcA;
    io.srcB = srcB;
    if (dA) {
      adp_bn_bwd_args a{};
      a.dA = dA;
      a.z = z;
      a.scale = stv(l, 2);
      a.shift = stv(l, 3);
      a.mean = stv(l, 4);
      a.invstd = stv(l, 5);
      a.gamma = P + l.offG;
      a.dgamma = G + l.offG;
      a.dbeta = G + l.offBeta;
      a.count = (float)((double)N * H * H);
      CL(adp_conv_wgrad_bn(cfg.dtype, &d, &io, &a, dz, l.cout_s, G + l.offW, nullptr, s));
    } else {
      CL(adp_conv_wgrad(cfg.dtype, &d, &io, dz, l.cout_s, G + l.offW, nullptr, s));
    }
    return ready(bl_idx.at(name), s);
  }
  int bn_backward(int N, hipStream_t s) {
    const int dt = cfg.dtype, Lv = levels;
    // data-gradient weights of every layer but the input conv and the head, batched
    std::vector<adp_pack_job> jobs;
    for (auto& l : bl) {
      if (!l.Wd) continue;
      adp_pack_job j{};
      j.src = P + l.offW;
      j.dst = l.Wd;
      j.taps = l.kind == 1 ? 1 : l.taps;
      j.Cin_s = l.Cin_s;
      j.Nout = l.kind == 1 ? l.Nout : l.cout_s;
      j.src_kpad = l.Kpad;
      j.dst_rows = l.dNpad;
      j.dst_kpad = l.dKpad;
      jobs.push_back(j);
    }
    for (size_t i = 0; i < jobs.size(); i += ADP_PACK_MAX_JOBS)
      CL(adp_pack_weights_batch(dt, (int)std::min<size_t>(ADP_PACK_MAX_JOBS, jobs.size() - i), jobs.data() + i, s));
    const size_t M0 = (size_t)N * S * S;
    BnLayer& h = L("head");
    BnLayer& l0 = L("dec0_conv2");
    // head backward with dec0_conv2's BatchNorm-backward reduction fused; dA is not stored (recomputed below)
    CL(adp_head_sigmoid_bwd_bnr(dt, M0, l0.cout_s, h.cin[0], b("y0_2"), P + h.offW, stv(l0, 2), stv(l0, 3),
                                stv(l0, 4), stv(l0, 5), b<float>("p"), b<float>("dp_main"), nullptr, G + h.offW,
                                G + h.offB, G + l0.offG, G + l0.offBeta, s));
    CL(ready(bl_idx.at("head"), s));
    CL(adp_fill_f32(n_stat_bwd, 0.f, stat_bwd, s));
    const void* cur_dA = nullptr;
    const void* bott_dA = nullptr;
    std::vector<void*> skip(Lv, nullptr);
    for (int i = 0; i < Lv - 1; ++i) {
      const std::string k = std::to_string(i), dn = "dec" + k;
      void* dz = b(("dz_y" + k + "_2").c_str());
      if (!cur_dA) {   // level 0: dA = dL/d relu(bn(y0_2)) recomputed from the head (bit-identical dz)
        CL(adp_bn_bwd_apply_head(dt, M0, l0.cout_s, h.cin[0], P + h.offW, b<float>("p"), b<float>("dp_main"),
                                 b("y0_2"), stv(l0, 2), stv(l0, 3), stv(l0, 4), stv(l0, 5), P + l0.offG, G + l0.offG,
                                 G + l0.offBeta, (float)M0, dz, s));
        CL(bn_wgrad(dn + "_conv2", N, b(("ay" + k + "_1").c_str()), nullptr, nullptr, nullptr, dz, s));
      } else {
        CL(bn_wgrad(dn + "_conv2", N, b(("ay" + k + "_1").c_str()), nullptr, cur_dA, b(("y" + k + "_2").c_str()), dz,
                    s));
      }
      void* dA1 = b(("dA_y" + k + "_1").c_str());
      CL(bn_dgrad(dn + "_conv2", N, dz, dA1, dn + "_conv1", b(("y" + k + "_1").c_str()), s));
      void* dz1 = b(("dz_y" + k + "_1").c_str());
      CL(bn_wgrad(dn + "_conv1", N, b(("az" + k + "_2").c_str()), b(("t" + k).c_str()), dA1, b(("y" + k + "_1").c_str()),
                  dz1, s));
      // concat data gradient split into the skip part and the ConvTranspose output part; the ConvTranspose
      // bias gradient is the epilogue channel sum of the second part
      BnLayer& l1 = L(dn + "_conv1");
      BnLayer& lu = L(dn + "_up");
      void* sk = b(("skip" + k).c_str());
      void* dtb = b(("dt" + k).c_str());
      {
        const int H = side(i);
        adp_conv_desc d = desc3(N, H, l1);
        d.CA_stride = l1.cout_s;
        d.CB_stride = 0;
        d.Nout = l1.Cin_s;
        d.out_mode = 2;
        d.out_stride = l1.cin_s[0];
        d.out2_stride = l1.cin_s[1];
        d.split_c = l1.cin_s[0];
        adp_conv_io io{};
        io.srcA = dz1;
        io.W = l1.Wd;
        io.out = sk;
        io.out2 = dtb;
        io.bn_sum = dtsum[i];
        io.bn_sqsum = dtsum[i] + l1.Cin_s;
        CL(adp_conv_fwd(dt, &d, &io, s));
      }
      CL(adp_ew_add_mask(ADP_DTYPE_F32, lu.cout_s, G + lu.offB, dtsum[i] + l1.cin_s[0], nullptr, 1.f, G + lu.offB, s));
      skip[i] = sk;
      const std::string pk = std::to_string(i + 1);
      const void* pact = i + 1 < Lv - 1 ? b(("ay" + pk + "_2").c_str()) : b(("az" + std::to_string(Lv - 1) + "_2").c_str());
      {
        adp_conv_desc d{};
        d.N = N;
        d.Hs = d.Ws = d.Ho = d.Wo = side(i + 1);
        d.CA_stride = lu.cin_s[0];
        d.stride = 1;
        d.kh = d.kw = 1;
        d.dil = 1;
        d.pad = 0;
        d.Nout = lu.Nout;
        d.out_mode = 1;
        d.shuffle_c = lu.cout_s;
        d.mask_scale = d.mask2_scale = 1.f;
        adp_conv_io io{};
        io.srcA = pact;
        CL(adp_conv_wgrad(dt, &d, &io, dtb, lu.cout_s, G + lu.offW, nullptr, s));
        CL(ready(bl_idx.at(lu.name), s));
      }
      void* dAp = b(("dA_up" + k).c_str());
      if (i + 1 < Lv - 1) {
        CL(convt_dgrad(lu.name, N, dtb, dAp, "dec" + pk + "_conv2", b(("y" + pk + "_2").c_str()), s));
        cur_dA = dAp;
      } else {
        CL(convt_dgrad(lu.name, N, dtb, dAp, "enc" + pk + "_conv2", b(("z" + pk + "_2").c_str()), s));
        bott_dA = dAp;
      }
    }
    // bottleneck + encoder, deepest level first
    const void* dpool = nullptr;
    for (int i = Lv - 1; i >= 0; --i) {
      const std::string k = std::to_string(i), en = "enc" + k;
      void* z2 = b(("z" + k + "_2").c_str());
      void* z1 = b(("z" + k + "_1").c_str());
      const void* dA2 = nullptr;
      if (i < Lv - 1) {   // pool backward (argmax recomputed from z) + skip gradient + fused BN-backward reduction
        BnLayer& r = L(en + "_conv2");
        void* d2 = b(("dA_z" + k + "_2").c_str());
        CL(adp_maxpool2_bwd_bnr(dt, N, side(i), side(i), r.cout_s, nullptr, dpool, skip[i], d2, z2, stv(r, 2), stv(r, 3),
                                stv(r, 4), stv(r, 5), G + r.offG, G + r.offBeta, s));
        dA2 = d2;
      } else {
        dA2 = Lv > 1 ? bott_dA : nullptr;
        if (!dA2) { adp::set_error("unet_bn handle: needs levels >= 2"); return -1; }
      }
      void* dz2 = b(("dz_z" + k + "_2").c_str());
      CL(bn_wgrad(en + "_conv2", N, b(("az" + k + "_1").c_str()), nullptr, dA2, z2, dz2, s));
      void* dA1 = b(("dA_z" + k + "_1").c_str());
      CL(bn_dgrad(en + "_conv2", N, dz2, dA1, en + "_conv1", z1, s));
      // (the input layer has no data gradient: its dz is not stored where the fused input-layer form runs, bf16
      // with 64 base channels; elsewhere the two-launch form writes it into the handle's own buffer)
      void* dz1 = (i == 0 && in_dz_fused()) ? nullptr : b(("dz_z" + k + "_1").c_str());
      const void* src = i == 0 ? b("x") : b(("pool" + std::to_string(i - 1)).c_str());
      CL(bn_wgrad(en + "_conv1", N, src, nullptr, dA1, z1, dz1, s));
      if (i > 0) {
        void* dp = b(("dpool" + std::to_string(i - 1)).c_str());
        CL(bn_dgrad(en + "_conv1", N, dz1, dp, "", nullptr, s));
        dpool = dp;
      }
    }
    return 0;
  }

  // -- Keras-layout parameter I/O of unet_bn (slot 0 kernel, conv+BN: 1 gamma, 2 beta, 3 moving mean,
  // 4 moving variance; ConvTranspose / head: 1 bias); synchronous
  size_t bn_param_size(const BnLayer& l, int slot) const {
    const size_t cin = l.kind == 2 ? l.cin[0] : (size_t)(l.cin.size() > 1 ? l.cin[0] + l.cin[1] : l.cin[0]);
    if (slot == 0) return l.kind == 0 ? 9 * cin * l.cout : (l.kind == 1 ? 4 * cin * l.cout : cin);
    if (l.kind == 0) return slot <= 4 ? (size_t)l.cout : 0;
    return slot == 1 ? (size_t)(l.kind == 2 ? 1 : l.cout) : 0;
  }
  std::vector<int> cmap(const BnLayer& l) const {
    std::vector<int> cm;
    int base_c = 0;
    for (size_t p = 0; p < l.cin.size(); ++p) {
      for (int c = 0; c < l.cin[p]; ++c) cm.push_back(base_c + c);
      base_c += l.cin_s[p];
    }
    return cm;
  }
  float* bn_slot_ptr(BnLayer& l, int slot) {
    if (l.kind == 0) {
      switch (slot) {
        case 1: return P + l.offG;
        case 2: return P + l.offBeta;
        case 3: return l.rmean;
        case 4: return l.rvar;
      }
      return nullptr;
    }
    return slot == 1 ? P + l.offB : nullptr;
  }
  int bn_set_param(BnLayer& l, int slot, const float* host) {
    CK(hipDeviceSynchronize());
    if (slot != 0) {
      CK(hipMemcpy(bn_slot_ptr(l, slot), host, sizeof(float) * bn_param_size(l, slot), hipMemcpyHostToDevice));
      return 0;
    }
    const std::vector<int> cm = cmap(l);
    const int cin = (int)cm.size();
    if (l.kind == 2) {
      std::vector<float> w(rup64(cin), 0.f);
      for (int c = 0; c < cin; ++c) w[c] = host[c];
      CK(hipMemcpy(P + l.offW, w.data(), sizeof(float) * cin, hipMemcpyHostToDevice));
      return 0;
    }
    std::vector<float> wp((size_t)l.Npad * l.Kpad, 0.f);
    if (l.kind == 0) {   // HWIO (3, 3, cin, cout) -> [co][t * Cin_s + cm[ci]]
      for (int t = 0; t < 9; ++t)
        for (int ci = 0; ci < cin; ++ci)
          for (int co = 0; co < l.cout; ++co)
            wp[(size_t)co * l.Kpad + t * l.Cin_s + cm[ci]] = host[((size_t)t * cin + ci) * l.cout + co];
    } else {             // torch ConvTranspose (cin, cout, 2, 2) -> [sub * cout_s + co][cm[ci]]
      for (int ci = 0; ci < cin; ++ci)
        for (int co = 0; co < l.cout; ++co)
          for (int sub = 0; sub < 4; ++sub)
            wp[(size_t)(sub * l.cout_s + co) * l.Kpad + cm[ci]] = host[((size_t)ci * l.cout + co) * 4 + sub];
    }
    CK(hipMemcpy(P + l.offW, wp.data(), sizeof(float) * wp.size(), hipMemcpyHostToDevice));
    return 0;
  }
  // src = P (parameters) or G (the last step's gradients; slots 3 / 4 have none)
  int bn_get_param(BnLayer& l, int slot, float* host, const float* src = nullptr) {
    CK(hipDeviceSynchronize());
    const bool grad = src == G;
    if (!src) src = P;
    if (slot != 0) {
      const float* p = bn_slot_ptr(l, slot);
      if (grad) {
        if (l.kind == 0 && slot >= 3) { adp::set_error("adp_get_grad: running statistics have no gradient"); return -1; }
        p = G + (p - P);
      }
      CK(hipMemcpy(host, p, sizeof(float) * bn_param_size(l, slot), hipMemcpyDeviceToHost));
      return 0;
    }
    const std::vector<int> cm = cmap(l);
    const int cin = (int)cm.size();
    if (l.kind == 2) {
      CK(hipMemcpy(host, src + l.offW, sizeof(float) * cin, hipMemcpyDeviceToHost));
      return 0;
    }
    std::vector<float> wp((size_t)l.Npad * l.Kpad);
    CK(hipMemcpy(wp.data(), src + l.offW, sizeof(float) * wp.size(), hipMemcpyDeviceToHost));
    if (l.kind == 0) {
      for (int t = 0; t < 9; ++t)
        for (int ci = 0; ci < cin; ++ci)
          for (int co = 0; co < l.cout; ++co)
            host[((size_t)t * cin + ci) * l.cout + co] = wp[(size_t)co * l.Kpad + t * l.Cin_s + cm[ci]];
    } else {
      for (int ci = 0; ci < cin; ++ci)
        for (int co = 0; co < l.cout; ++co)
          for (int sub = 0; sub < 4; ++sub)
            host[((size_t)ci * l.cout + co) * 4 + sub] = wp[(size_t)(sub * l.cout_s + co) * l.Kpad + cm[ci]];
    }
    return 0;
  }
};

extern "C" int adp_create(const adp_config* cfg, int device, adp_handle** out) {
  if (!cfg || !out) { adp::set_error("adp_create: null argument"); return -1; }
  *out = nullptr;
  if (cfg->preset != ADP_PRESET_ADIPOSE_V3 && cfg->preset != ADP_PRESET_UNET_BN) {
    adp::set_error("adp_create: preset ADP_PRESET_ADIPOSE_V3 or ADP_PRESET_UNET_BN");
    return -1;
  }
  if (cfg->tile <= 0 || cfg->tile % 8 || cfg->max_batch <= 0 ||
      (cfg->dtype != ADP_DTYPE_F32 && cfg->dtype != ADP_DTYPE_BF16)) {
    adp::set_error("adp_create: tile % 8 == 0, max_batch > 0, dtype f32 or bf16");
    return -1;
  }
  if (cfg->dropout_rate < 0.f || cfg->dropout_rate >= 1.f) {
    adp::set_error("adp_create: dropout_rate in [0, 1)");
    return -1;
  }
  if (cfg->preset == ADP_PRESET_UNET_BN) {
    const int lv = cfg->levels > 0 ? cfg->levels : 5, bs = cfg->base > 0 ? cfg->base : 64;
    const int ic = cfg->in_ch > 0 ? cfg->in_ch : 3;
    if (lv < 2 || lv > 8 || cfg->tile % (1 << (lv - 1)) || bs % 8 || ic > 8 || (bs << (lv - 1)) > 2048) {
      adp::set_error("adp_create(unet_bn): 2 <= levels <= 8, tile divisible by 2^(levels-1), base % 8 == 0, "
                     "in_ch <= 8, base << (levels-1) <= 2048");
      return -1;
    }
    if (hipSetDevice(device) != hipSuccess) { adp::set_error("adp_create: hipSetDevice failed"); return -2; }
    auto* h = new adp_handle();
    h->cfg = *cfg;
    h->device = device;
    h->S = cfg->tile;
    h->B = cfg->max_batch;
    h->es = cfg->dtype == ADP_DTYPE_F32 ? 4 : 2;
    h->levels = lv;
    h->base = bs;
    h->in_ch = ic;
    const int rc = h->create_unet_bn();
    if (rc) { delete h; return rc; }
    *out = h;
    return 0;
  }
  if (hipSetDevice(device) != hipSuccess) { adp::set_error("adp_create: hipSetDevice failed"); return -2; }
  auto* h = new adp_handle();
  h->cfg = *cfg;
  h->device = device;
  h->S = cfg->tile;
  h->B = cfg->max_batch;
  h->nb = cfg->init_nb > 0 ? cfg->init_nb : 44;
  h->es = cfg->dtype == ADP_DTYPE_F32 ? 4 : 2;
  // channel layout of nets.AdiposeV3Net: bf16 64/128/192/384 (predictor.INFER_CPAD), f32 64/96/192/352
  for (int i = 0; i < 4; ++i) h->cpad[i] = cfg->dtype == ADP_DTYPE_BF16 ? 64 : 32;
  const int nb = h->nb;
  for (int i = 0; i < 4; ++i) {
    h->ch[i] = round_up((1 << i) * nb, h->cpad[i]);
    h->sz[i] = h->S >> i;
  }
  h->add_dense("down1_conv1", -1, {1}, 0, nb);
  h->add_dense("down1_conv2", 0, {nb}, 0, nb);
  h->add_dense("down2_conv1", 0, {nb}, 1, 2 * nb);
  h->add_dense("down2_conv2", 1, {2 * nb}, 1, 2 * nb);
  h->add_dense("down3_conv1", 1, {2 * nb}, 2, 4 * nb);
  h->add_dense("down3_conv2", 2, {4 * nb}, 2, 4 * nb);
  const int dils[6] = {1, 2, 4, 8, 16, 32};
  for (int i = 0; i < 6; ++i) {
    const std::string n = "dilate" + std::to_string(i + 1);
    h->add_dense(n.c_str(), i == 0 ? 2 : 3, {i == 0 ? 4 * nb : 8 * nb}, 3, 8 * nb, dils[i]);
  }
  h->add_dense("up3_conv1", 3, {8 * nb}, 2, 4 * nb, 1, 1);
  h->add_dense("up3_conv2", 2, {4 * nb, 4 * nb}, 2, 4 * nb);
  h->add_dense("up3_conv3", 2, {4 * nb}, 2, 4 * nb);
  h->add_dense("up2_conv1", 2, {4 * nb}, 1, 2 * nb, 1, 1);
  h->add_dense("up2_conv2", 1, {2 * nb, 2 * nb}, 1, 2 * nb);
  h->add_dense("up2_conv3", 1, {2 * nb}, 1, 2 * nb);
  h->add_dense("up1_conv1", 1, {2 * nb}, 0, nb, 1, 1);
  h->add_dense("up1_conv2", 0, {nb, nb}, 0, nb);
  h->add_dense("up1_conv3", 0, {nb}, 0, nb);
  if (cfg->deep_supervision) {   // loaded for checkpoint compatibility; inference returns main_out
    h->add_head("aux_out1", 4 * nb, 1, 2);
    h->add_head("aux_out2", 2 * nb, 1, 1);
  }
  h->add_head("output_softmax", nb, 2, 0);

  auto fail = [&](int rc) { delete h; return rc; };
  size_t wmax = 0;
  for (auto& l : h->dense) {
    if (hipMalloc(&l.W, (size_t)l.Npad * l.Kpad * h->es) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&l.b), sizeof(float) * l.cout_s) != hipSuccess) {
      adp::set_error("adp_create: weight allocation failed");
      return fail(-2);
    }
    (void)hipMemset(l.W, 0, (size_t)l.Npad * l.Kpad * h->es);
    wmax = std::max(wmax, (size_t)l.Npad * l.Kpad);
  }
  for (auto& hd : h->heads)
    if (hipMalloc(reinterpret_cast<void**>(&hd.W), sizeof(float) * hd.cin * hd.nout) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&hd.b), sizeof(float) * hd.nout) != hipSuccess) {
      adp::set_error("adp_create: head allocation failed");
      return fail(-2);
    }
  if (cfg->dtype != ADP_DTYPE_F32 && hipMalloc(reinterpret_cast<void**>(&h->wstage), sizeof(float) * wmax) != hipSuccess) {
    adp::set_error("adp_create: staging allocation failed");
    return fail(-2);
  }
  // activations for B images: the buffers of nets.AdiposeV3Net.alloc
  const size_t B = h->B, es = h->es;
  auto act = [&](const char* n, int lvl, int cidx) {
    return h->alloc(n, B * h->sz[lvl] * h->sz[lvl] * h->ch[cidx] * es);
  };
  int rc = h->alloc("x", B * h->S * h->S * 8 * es);
  const char* per_level[3][3] = {{"d1a", "d1", "p1"}, {"d2a", "d2", "p2"}, {"d3a", "d3", "p3"}};
  for (int l = 0; l < 3 && !rc; ++l) {
    rc = rc || act(per_level[l][0], l, l) || act(per_level[l][1], l, l) || act(per_level[l][2], l + 1, l);
  }
  for (int i = 1; i <= 6 && !rc; ++i) rc = act(("dl" + std::to_string(i)).c_str(), 3, 3);
  if (!rc && cfg->dtype == ADP_DTYPE_F32) rc = h->alloc("dsum_f", B * h->sz[3] * h->sz[3] * h->ch[3] * 4);
  if (!rc && cfg->dtype != ADP_DTYPE_F32) rc = act("dsum", 3, 3);
  const char* ups[3][3] = {{"u3a", "u3b", "u3"}, {"u2a", "u2b", "u2"}, {"u1a", "u1b", "u1"}};
  for (int u = 0; u < 3 && !rc; ++u)
    for (int j = 0; j < 3 && !rc; ++j) rc = act(ups[u][j], 2 - u, 2 - u);
  if (!rc) rc = h->alloc("p_main", B * h->S * h->S * 4);
  if (!rc) rc = h->alloc("probs", B * h->S * h->S * 4);
  if (rc) return fail(rc);
  *out = h;
  return 0;
}

extern "C" int adp_destroy(adp_handle* h) {
  delete h;
  return 0;
}

extern "C" const char* adp_param_name(const adp_handle* h, int i) {
  if (!h || i < 0) return nullptr;
  if (!h->bl.empty()) return i < (int)h->bl.size() ? h->bl[i].name.c_str() : nullptr;
  if (i < (int)h->dense.size()) return h->dense[i].name.c_str();
  i -= (int)h->dense.size();
  return i < (int)h->heads.size() ? h->heads[i].name.c_str() : nullptr;
}

static std::vector<float>* param_ref(adp_handle* h, const char* layer, int slot) {
  if (!h || !layer || (slot != 0 && slot != 1)) return nullptr;
  auto d = h->dense_idx.find(layer);
  if (d != h->dense_idx.end()) return slot == 0 ? &h->dense[d->second].kernel : &h->dense[d->second].bias;
  auto e = h->head_idx.find(layer);
  if (e != h->head_idx.end()) return slot == 0 ? &h->heads[e->second].kernel : &h->heads[e->second].bias;
  return nullptr;
}

// unet_bn handles: the layer, or nullptr (error set) for an unknown name / slot
static BnLayer* bn_param(adp_handle* h, const char* layer, int slot, const char* who) {
  auto it = h->bl_idx.find(layer ? layer : "");
  if (it == h->bl_idx.end() || slot < 0 || h->bn_param_size(h->bl[it->second], slot) == 0) {
    adp::set_error(std::string(who) + ": unknown unet_bn parameter " + (layer ? layer : "(null)") + " slot " +
                   std::to_string(slot) + " (conv: 0 kernel, 1 gamma, 2 beta, 3 moving mean, 4 moving variance; "
                   "ConvTranspose / head: 0 kernel, 1 bias)");
    return nullptr;
  }
  return &h->bl[it->second];
}

extern "C" int adp_param_size(adp_handle* h, const char* layer, int slot, size_t* n) {
  if (h && !h->bl.empty()) {
    BnLayer* l = bn_param(h, layer, slot, "adp_param_size");
    if (!l || !n) return -1;
    *n = h->bn_param_size(*l, slot);
    return 0;
  }
  std::vector<float>* v = param_ref(h, layer, slot);
  if (!v || !n) { adp::set_error(std::string("adp_param_size: unknown parameter ") + (layer ? layer : "(null)")); return -1; }
  *n = v->size();
  return 0;
}

extern "C" int adp_set_param(adp_handle* h, const char* layer, int slot, const float* host, size_t n) {
  if (h && !h->bl.empty()) {
    BnLayer* l = bn_param(h, layer, slot, "adp_set_param");
    if (!l) return -1;
    if (!host || n != h->bn_param_size(*l, slot)) {
      adp::set_error("adp_set_param: " + std::string(layer) + " slot " + std::to_string(slot) + " expects " +
                     std::to_string(h->bn_param_size(*l, slot)) + " floats");
      return -1;
    }
    if (hipSetDevice(h->device) != hipSuccess) { adp::set_error("adp_set_param: hipSetDevice failed"); return -2; }
    return h->bn_set_param(*l, slot, host);
  }
  std::vector<float>* v = param_ref(h, layer, slot);
  if (!v) { adp::set_error(std::string("adp_set_param: unknown parameter ") + (layer ? layer : "(null)")); return -1; }
  if (!host || n != v->size()) {
    adp::set_error("adp_set_param: " + std::string(layer) + " expects " + std::to_string(v->size()) + " floats");
    return -1;
  }
  if (h->host_stale) CL(h->download());   // the other layers' host copies must hold the trained values
  std::memcpy(v->data(), host, n * sizeof(float));
  h->dirty = true;
  return 0;
}

extern "C" int adp_get_param(adp_handle* h, const char* layer, int slot, float* host, size_t n) {
  if (h && !h->bl.empty()) {
    BnLayer* l = bn_param(h, layer, slot, "adp_get_param");
    if (!l) return -1;
    if (!host || n != h->bn_param_size(*l, slot)) { adp::set_error("adp_get_param: size mismatch"); return -1; }
    if (hipSetDevice(h->device) != hipSuccess) { adp::set_error("adp_get_param: hipSetDevice failed"); return -2; }
    return h->bn_get_param(*l, slot, host);
  }
  std::vector<float>* v = param_ref(h, layer, slot);
  if (!v || !host || n != v->size()) { adp::set_error("adp_get_param: unknown parameter or size mismatch"); return -1; }
  if (h->host_stale) {
    if (hipDeviceSynchronize() != hipSuccess) { adp::set_error("adp_get_param: device error"); return -2; }
    CL(h->download());
  }
  std::memcpy(host, v->data(), n * sizeof(float));
  return 0;
}

extern "C" int adp_get_grad(adp_handle* h, const char* layer, int slot, float* host, size_t n) {
  if (!h || !host) { adp::set_error("adp_get_grad: null argument"); return -1; }
  if (!h->train_on || !h->G || h->step == 0) { adp::set_error("adp_get_grad: no training step has run"); return -1; }
  if (hipSetDevice(h->device) != hipSuccess) { adp::set_error("adp_get_grad: hipSetDevice failed"); return -2; }
  if (!h->bl.empty()) {
    BnLayer* l = bn_param(h, layer, slot, "adp_get_grad");
    if (!l) return -1;
    if (n != h->bn_param_size(*l, slot)) { adp::set_error("adp_get_grad: size mismatch"); return -1; }
    return h->bn_get_param(*l, slot, host, h->G);
  }
  std::vector<float>* v = param_ref(h, layer, slot);
  if (!v || n != v->size()) { adp::set_error("adp_get_grad: unknown parameter or size mismatch"); return -1; }
  return h->v3_get_grad(layer, slot, host);
}

extern "C" int adp_debug_grad_flat(adp_handle* h, int which, float* host, size_t n) {
  if (!h || (which != 0 && which != 1)) { adp::set_error("adp_debug_grad_flat: bad arguments (which 0 or 1)"); return -1; }
  if (!h->train_on || !h->G || h->step == 0) { adp::set_error("adp_debug_grad_flat: no training step has run"); return -1; }
  if (n != h->nflat || !host) {
    adp::set_error("adp_debug_grad_flat: n must be the flat gradient size " + std::to_string(h->nflat));
    return -1;
  }
  const float* src = which == 0 ? h->G : h->Gsnap;
  if (!src) { adp::set_error("adp_debug_grad_flat: no snapshot (set option dp_snapshot = 1, train with a communicator)"); return -1; }
  if (hipSetDevice(h->device) != hipSuccess) { adp::set_error("adp_debug_grad_flat: hipSetDevice failed"); return -2; }
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(host, src, sizeof(float) * n, hipMemcpyDeviceToHost));
  return 0;
}

extern "C" int adp_forward(adp_handle* h, const float* images, int n, long long img_stride, float mean, float std_,
                           int tta_mode, float* prob, adp_stream_t st) {
  if (!h || !images || !prob || n < 0 || tta_mode < 0 || tta_mode > 3) {
    adp::set_error("adp_forward: bad arguments (tta_mode 0 none, 1 minimal, 2 basic, 3 full)");
    return -1;
  }
  hipStream_t s = (hipStream_t)st;
  if (hipSetDevice(h->device) != hipSuccess) { adp::set_error("adp_forward: hipSetDevice failed"); return -2; }
  const bool bn = !h->bl.empty();
  if (!bn && h->dirty) CL(h->upload(s));
  if (!bn && h->wpack_stale) CL(h->pack_forward(s));
  const int cin = bn ? h->in_ch : 1;   // unet_bn tiles: (S, S, in_ch) interleaved
  static const int views_tab[4][8] = {{0}, {0, 4}, {0, 4, 5, 1}, {0, 1, 2, 3, 4, 5, 6, 7}};
  static const int nviews[4] = {1, 2, 4, 8};
  const int nv = nviews[tta_mode];
  const int* views = views_tab[tta_mode];
  const int S = h->S;
  const size_t plane = (size_t)S * S;
  const long long istride = img_stride > 0 ? img_stride : (long long)plane * cin;
  const int per = std::max(1, h->B / nv);
  for (int i0 = 0; i0 < n; i0 += per) {
    const int cnt = std::min(per, n - i0), N = cnt * nv;
    if (N > h->B) { adp::set_error("adp_forward: TTA views exceed max_batch"); return -1; }
    for (int t = 0; t < cnt; ++t)
      for (int k = 0; k < nv; ++k)
        CL(adp_prep_input(h->cfg.dtype, 1, S, S, cin, images + (size_t)(i0 + t) * istride, S, (long long)plane * cin,
                          mean, std_, views[k], 8,
                          static_cast<char*>(h->b("x")) + (size_t)(t * nv + k) * plane * 8 * h->es, s));
    if (bn) CL(h->bn_forward(N, false, s));
    else CL(h->forward(N, s));
    for (int t = 0; t < cnt; ++t) {
      const float* p = h->b<float>(bn ? "p" : "p_main") + (size_t)t * nv * plane;
      if (nv == 1) CL(adp_cast(ADP_DTYPE_F32, ADP_DTYPE_F32, plane, p, prob + (size_t)(i0 + t) * plane, s));
      else CL(adp_tta_merge(S, S, nv, views, p, prob + (size_t)(i0 + t) * plane, s));
    }
  }
  return 0;
}

extern "C" int adp_set_comm(adp_handle* h, void* comm) {
  if (!h) { adp::set_error("adp_set_comm: null handle"); return -1; }
  if (comm && !rccl().ok) { adp::set_error("adp_set_comm: librccl.so.1 not loadable"); return -3; }
  h->comm = comm;
  // (the persistent kernels keep their static tile lists under data parallelism: in the bucket schedule a held
  // CU frees within one bucket's all-reduce, and static lists measured cheaper than claimed tiles end to end --
  // DESIGN.md §5, profiles/r04c_bucket_probe.log; option dp_claim=1 turns claiming on)
  return 0;
}

extern "C" int adp_comm_unique_id(void* id128) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId");
  if (!id128) { adp::set_error("adp_comm_unique_id: null"); return -1; }
  if (!rccl().ok) { adp::set_error("adp_comm_unique_id: librccl.so.1 not loadable"); return -3; }
  ncclUniqueId id;
  NC(rccl().get_id(&id));
  std::memcpy(id128, &id, sizeof(id));
  return 0;
}

extern "C" int adp_comm_init(int nranks, const void* id128, int rank, void** comm) {
  if (!id128 || !comm || nranks < 1 || rank < 0 || rank >= nranks) { adp::set_error("adp_comm_init: bad arguments"); return -1; }
  if (!rccl().ok) { adp::set_error("adp_comm_init: librccl.so.1 not loadable"); return -3; }
  ncclUniqueId id;
  std::memcpy(&id, id128, sizeof(id));
  ncclComm_t c = nullptr;
  NC(rccl().init(&c, nranks, id, rank));
  *comm = c;
  return 0;
}

extern "C" int adp_comm_destroy(void* comm) {
  if (!comm) return 0;
  if (!rccl().ok) { adp::set_error("adp_comm_destroy: librccl.so.1 not loadable"); return -3; }
  NC(rccl().destroy(static_cast<ncclComm_t>(comm)));
  return 0;
}

extern "C" int adp_train_step(adp_handle* h, const float* x, const float* y, int n, const adp_train_cfg* cfg, float lr,
                              float* metrics, adp_stream_t st) {
  if (!h || !x || !y || !cfg || n <= 0) { adp::set_error("adp_train_step: bad arguments"); return -1; }
  if (n > h->B) { adp::set_error("adp_train_step: n exceeds max_batch"); return -1; }
  if (cfg->dropout_rate >= 1.f || cfg->hard_example_ratio <= 0.f || cfg->hard_example_ratio > 1.f) {
    adp::set_error("adp_train_step: dropout_rate < 1 (< 0: the model's build_model rate), hard_example_ratio in (0, 1]");
    return -1;
  }
  const bool bn = !h->bl.empty();
  if (bn && cfg->freeze_encoder) {
    adp::set_error("adp_train_step: the unet_bn preset has no frozen-encoder phase");
    return -1;
  }
  hipStream_t s = (hipStream_t)st;
  if (hipSetDevice(h->device) != hipSuccess) { adp::set_error("adp_train_step: hipSetDevice failed"); return -2; }
  CL(adp_bn_fold_reset(st));   // a failed earlier step may have left a deferred BatchNorm fold pending
  if (!bn) {
    CL(h->ensure_train());
    if (h->dirty) CL(h->upload(s));
    CL(h->pack_forward(s));
  }
  const int S = h->S, N = n;
  const size_t plane = (size_t)S * S;
  int world = 1;
  ncclComm_t comm = static_cast<ncclComm_t>(h->comm);
  if (comm) NC(rccl().count(comm, &world));
  // forward (Trainer.train_step: prep_input(x, mean 0, std 1), iterations += 1, forward(train, seed))
  const int cin = bn ? h->in_ch : 1;
  CL(adp_prep_input(h->cfg.dtype, N, S, S, cin, x, S, (long long)plane * cin, 0.f, 1.f, 0, 8, h->b("x"), s));
  h->step += 1;
  float keep = 1.f;
  if (bn) {
    CL(h->bn_forward(N, true, s));
  } else {
    const float r = cfg->dropout_rate >= 0.f ? cfg->dropout_rate : h->cfg.dropout_rate;
    keep = r > 0.f ? (float)(1.0 / (1.0 - (double)r)) : 1.f;
    const unsigned sd =
        (unsigned)((unsigned long long)((long long)(h->cfg.seed + (unsigned)h->step) * 7919 + 17) & 0xFFFFFFFFull);
    CL(h->forward(N, s, true, r, sd));
  }
  // losses and dL/dp (Trainer.loss_and_grads)
  const bool ds = !bn && h->cfg.deep_supervision != 0;
  struct Spec { const char* p; const char* dp; float w; int ohem; };
  std::vector<Spec> specs = {{bn ? "p" : "p_main", "dp_main", ds ? cfg->w_main : 1.f, cfg->use_hard_mining}};
  if (ds) {
    specs.push_back({"p_aux1", "dp_aux1", cfg->w_aux1, 0});
    specs.push_back({"p_aux2", "dp_aux2", cfg->w_aux2, 0});
  }
  double* stats = h->b<double>("stats");
  double* lossbuf = h->b<double>("lossbuf");
  float* rows = h->b<float>("rows");
  float* coef = h->b<float>("coef");
  CL(adp_fill_f32(3 * 8 * 2, 0.f, reinterpret_cast<float*>(stats), s));
  CL(adp_fill_f32(4 * 2, 0.f, reinterpret_cast<float*>(lossbuf), s));
  for (size_t i = 0; i < specs.size(); ++i)
    CL(adp_loss_rows(N, S, S, h->b<float>(specs[i].p), y, cfg->use_label_smoothing, cfg->epsilon_pos,
                     cfg->epsilon_neg, rows + i * (size_t)N * S, stats + 8 * i, s));
  // batch-global Dice sums (train_adipose_unet_v3.py:217-225) before the gradient
  if (comm) NC(rccl().allreduce(stats, stats, 24, ncclFloat64, ncclSum, comm, s));
  for (size_t i = 0; i < specs.size(); ++i) {
    const int k = specs[i].ohem ? (int)((float)S * cfg->hard_example_ratio) : S;
    CL(adp_loss_select(N, S, S, rows + i * (size_t)N * S, specs[i].ohem, cfg->hard_example_ratio, specs[i].w,
                       (float)((double)world * N * k), coef + i * (size_t)N * S, lossbuf + i, s));
    CL(adp_loss_grad(N, S, S, h->b<float>(specs[i].p), y, cfg->use_label_smoothing, cfg->epsilon_pos,
                     cfg->epsilon_neg, coef + i * (size_t)N * S, stats + 8 * i, specs[i].w, 0,
                     h->b<float>(specs[i].dp), s));
  }
  // backward with the bucketed gradient all-reduce overlapped, then Adam / AdamW over the trainable range
  CL(adp_fill_f32(h->nflat, 0.f, h->G, s));
  const bool full = !cfg->freeze_encoder;
  std::set<int> frozen;
  if (!full)
    for (const char* e : {"down1_conv1", "down1_conv2", "down2_conv1", "down2_conv2", "down3_conv1", "down3_conv2"})
      frozen.insert(h->dense_id(e));
  CL(h->dp_begin(frozen));
  // the deterministic weight-gradient reductions of the backward are recorded and launched together (adp_wgrad_defer:
  // one launch instead of ~21 with their dependency gaps); a bucket's all-reduce flushes first (dp_launch)
  CL(adp_wgrad_defer(1, s));
  h->deferring = true;
  const int brc = bn ? h->bn_backward(N, s) : h->backward(N, keep, full, s);
  h->deferring = false;
  const int frc = adp_wgrad_flush(s);
  if (brc || frc) {
    h->dp_abort(s);
    return brc ? brc : frc;
  }
  CL(h->dp_finish(s));
  const size_t lo = full ? 0 : h->enc_end;
  CL(adp_adam(h->nflat - lo, h->P + lo, h->G + lo, h->Mo + lo, h->Vo + lo, lr, cfg->beta1, cfg->beta2, cfg->eps, h->step,
              cfg->optimizer == 1 ? cfg->weight_decay : 0.f, 1.f, s));
  if (!bn) {
    h->host_stale = true;
    h->wpack_stale = h->cfg.dtype != ADP_DTYPE_F32;
  }
  if (!metrics) return 0;
  // Trainer.read_metrics (host read-back, synchronises)
  if (comm) NC(rccl().allreduce(lossbuf, lossbuf, 4, ncclFloat64, ncclSum, comm, s));
  double hs[24], hl[4];
  CK(hipMemcpyAsync(hs, stats, sizeof(hs), hipMemcpyDeviceToHost, s));
  CK(hipMemcpyAsync(hl, lossbuf, sizeof(hl), hipMemcpyDeviceToHost, s));
  CK(hipStreamSynchronize(s));
  double total = 0.0;
  float out[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (size_t i = 0; i < specs.size(); ++i) {
    const double* st_ = hs + 8 * i;
    const double dice = 1.0 - (2 * st_[0] + 1) / (st_[1] + st_[2] + 1);
    const double li = specs[i].w != 0.f ? hl[i] / specs[i].w + dice : 0.0;
    out[1 + i] = (float)li;
    total += specs[i].w * li;
  }
  out[0] = (float)total;
  out[4] = (float)((2 * hs[3] + 1) / (hs[4] + hs[5] + 1));
  out[5] = (float)(hs[6] / ((double)N * S * S * world));
  std::memcpy(metrics, out, sizeof(out));
  return 0;
}
