// Handle-level C ABI: a native adipose_v3 inference engine for non-Python callers.
//
//   adp_create(cfg, device, &h)          topology of AdiposeUNetV3.build_model (train_adipose_unet_v3.py:660-758,
//                                         segmentation_inference.py:88-146) at tile S, activation buffers for
//                                         cfg->max_batch images x TTA views, allocated once
//   adp_set_param / adp_get_param         Keras layer names and layouts (kernel HWIO, bias), so a
//                                         .weights.h5 maps 1:1 (slot 0 kernel, 1 bias)
//   adp_forward(h, images, n, ...)        predict_single (segmentation_inference.py:153-158) with optional
//                                         TTA (:181-229): z-score + view transform on load, all views of a
//                                         tile batched in one forward, inverse views averaged
//   adp_train_step(h, x, y, n, cfg, lr)   one model.net.fit step (train_adipose_unet_v3.py:1316-1324): forward
//                                         with dropout, OHEM / BCE+Dice / deep-supervision losses
//                                         (:217-363, :780-879), backward, [RCCL SUM all-reduce], Adam/AdamW
//   adp_set_comm / adp_comm_*             data parallel over an RCCL communicator (loaded at run time)
//   adp_destroy(h)
//
// The engine is host code over the library's own launchers (adp_conv_fwd, adp_maxpool2_fwd,
// adp_head_*_fwd, adp_prep_input, adp_tta_merge): the same kernels and schedule as nets.AdiposeV3Net.
// One handle per device and thread; calls are stream-ordered on the caller's stream (weights are
// uploaded synchronously by the first adp_forward after an adp_set_param).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>   // types and enums only: RCCL itself is loaded with dlopen

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/adipose_hip.h"

namespace adp {
void set_error(const std::string& msg);
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

  ~adp_handle() {
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
    d.mask_scale = d.mask2_scale = 1.f;
    io.srcA = srcA;
    io.srcB = srcB;
    return adp_conv_wgrad(cfg.dtype, &d, &io, dZ, l.cout_s, G + l.offW, G + l.offB, s);
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
    d.mask_scale = mscale;
    d.mask2_scale = 1.f;
    io.srcA = dZ;
    io.W = l.Wd;
    int ostride = l.Cin_s;
    if (skip_first) {
      io.W = static_cast<const char*>(l.Wd) + (size_t)l.cin_s[0] * l.dKpad * es;
      d.Nout = l.cin_s[1];
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
};

extern "C" int adp_create(const adp_config* cfg, int device, adp_handle** out) {
  if (!cfg || !out) { adp::set_error("adp_create: null argument"); return -1; }
  *out = nullptr;
  if (cfg->preset != ADP_PRESET_ADIPOSE_V3) { adp::set_error("adp_create: only ADP_PRESET_ADIPOSE_V3"); return -1; }
  if (cfg->tile <= 0 || cfg->tile % 8 || cfg->max_batch <= 0 ||
      (cfg->dtype != ADP_DTYPE_F32 && cfg->dtype != ADP_DTYPE_BF16)) {
    adp::set_error("adp_create: tile % 8 == 0, max_batch > 0, dtype f32 or bf16");
    return -1;
  }
  if (hipSetDevice(device) != hipSuccess) { adp::set_error("adp_create: hipSetDevice failed"); return -2; }
  auto* h = new adp_handle();
  h->cfg = *cfg;
  h->device = device;
  h->S = cfg->tile;
  h->B = cfg->max_batch;
  h->nb = cfg->init_nb > 0 ? cfg->init_nb : 44;
  h->es = cfg->dtype == ADP_DTYPE_F32 ? 4 : 2;
  if (cfg->dtype == ADP_DTYPE_BF16) {   // channel layout of predictor.INFER_CPAD: 64/128/192/384
    const int cp[4] = {64, 64, 64, 64};
    for (int i = 0; i < 4; ++i) h->cpad[i] = cp[i];
  }
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

extern "C" int adp_param_size(adp_handle* h, const char* layer, int slot, size_t* n) {
  std::vector<float>* v = param_ref(h, layer, slot);
  if (!v || !n) { adp::set_error(std::string("adp_param_size: unknown parameter ") + (layer ? layer : "(null)")); return -1; }
  *n = v->size();
  return 0;
}

extern "C" int adp_set_param(adp_handle* h, const char* layer, int slot, const float* host, size_t n) {
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
  std::vector<float>* v = param_ref(h, layer, slot);
  if (!v || !host || n != v->size()) { adp::set_error("adp_get_param: unknown parameter or size mismatch"); return -1; }
  if (h->host_stale) {
    if (hipDeviceSynchronize() != hipSuccess) { adp::set_error("adp_get_param: device error"); return -2; }
    CL(h->download());
  }
  std::memcpy(host, v->data(), n * sizeof(float));
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
  if (h->dirty) CL(h->upload(s));
  if (h->wpack_stale) CL(h->pack_forward(s));
  static const int views_tab[4][8] = {{0}, {0, 4}, {0, 4, 5, 1}, {0, 1, 2, 3, 4, 5, 6, 7}};
  static const int nviews[4] = {1, 2, 4, 8};
  const int nv = nviews[tta_mode];
  const int* views = views_tab[tta_mode];
  const int S = h->S;
  const size_t plane = (size_t)S * S;
  const long long istride = img_stride > 0 ? img_stride : (long long)plane;
  const int per = std::max(1, h->B / nv);
  for (int i0 = 0; i0 < n; i0 += per) {
    const int cnt = std::min(per, n - i0), N = cnt * nv;
    if (N > h->B) { adp::set_error("adp_forward: TTA views exceed max_batch"); return -1; }
    for (int t = 0; t < cnt; ++t)
      for (int k = 0; k < nv; ++k)
        CL(adp_prep_input(h->cfg.dtype, 1, S, S, 1, images + (size_t)(i0 + t) * istride, S, (long long)plane, mean,
                          std_, views[k], 8, static_cast<char*>(h->b("x")) + (size_t)(t * nv + k) * plane * 8 * h->es,
                          s));
    CL(h->forward(N, s));
    for (int t = 0; t < cnt; ++t) {
      const float* p = h->b<float>("p_main") + (size_t)t * nv * plane;
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
  if (cfg->dropout_rate < 0.f || cfg->dropout_rate >= 1.f || cfg->hard_example_ratio <= 0.f ||
      cfg->hard_example_ratio > 1.f) {
    adp::set_error("adp_train_step: dropout_rate in [0, 1), hard_example_ratio in (0, 1]");
    return -1;
  }
  hipStream_t s = (hipStream_t)st;
  if (hipSetDevice(h->device) != hipSuccess) { adp::set_error("adp_train_step: hipSetDevice failed"); return -2; }
  CL(h->ensure_train());
  if (h->dirty) CL(h->upload(s));
  CL(h->pack_forward(s));
  const int S = h->S, N = n;
  const size_t plane = (size_t)S * S;
  int world = 1;
  ncclComm_t comm = static_cast<ncclComm_t>(h->comm);
  if (comm) NC(rccl().count(comm, &world));
  // forward (Trainer.train_step: prep_input(x, mean 0, std 1), iterations += 1, forward(train, seed))
  CL(adp_prep_input(h->cfg.dtype, N, S, S, 1, x, S, (long long)plane, 0.f, 1.f, 0, 8, h->b("x"), s));
  h->step += 1;
  const float r = cfg->dropout_rate;
  const float keep = r > 0.f ? (float)(1.0 / (1.0 - (double)r)) : 1.f;
  const unsigned sd = (unsigned)((unsigned long long)((long long)h->step * 7919 + 17) & 0xFFFFFFFFull);
  CL(h->forward(N, s, true, r, sd));
  // losses and dL/dp (Trainer.loss_and_grads)
  const bool ds = h->cfg.deep_supervision != 0;
  struct Spec { const char* p; const char* dp; float w; int ohem; };
  std::vector<Spec> specs = {{"p_main", "dp_main", ds ? cfg->w_main : 1.f, cfg->use_hard_mining}};
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
  if (comm) NC(rccl().allreduce(stats, stats, 24, ncclFloat64, ncclSum, comm, s));
  for (size_t i = 0; i < specs.size(); ++i) {
    const int k = specs[i].ohem ? (int)((float)S * cfg->hard_example_ratio) : S;
    CL(adp_loss_select(N, S, S, rows + i * (size_t)N * S, specs[i].ohem, cfg->hard_example_ratio, specs[i].w,
                       (float)((double)world * N * k), coef + i * (size_t)N * S, lossbuf + i, s));
    CL(adp_loss_grad(N, S, S, h->b<float>(specs[i].p), y, cfg->use_label_smoothing, cfg->epsilon_pos,
                     cfg->epsilon_neg, coef + i * (size_t)N * S, stats + 8 * i, specs[i].w, 0,
                     h->b<float>(specs[i].dp), s));
  }
  // backward, gradient all-reduce, Adam / AdamW over the trainable part of the flat buffer
  CL(adp_fill_f32(h->nflat, 0.f, h->G, s));
  const bool full = !cfg->freeze_encoder;
  CL(h->backward(N, keep, full, s));
  if (comm) NC(rccl().allreduce(h->G, h->G, h->nflat, ncclFloat32, ncclSum, comm, s));
  const size_t lo = full ? 0 : h->enc_end;
  CL(adp_adam(h->nflat - lo, h->P + lo, h->G + lo, h->Mo + lo, h->Vo + lo, lr, cfg->beta1, cfg->beta2, cfg->eps, h->step,
              cfg->optimizer == 1 ? cfg->weight_decay : 0.f, 1.f, s));
  h->host_stale = true;
  h->wpack_stale = h->cfg.dtype != ADP_DTYPE_F32;
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
