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
//   adp_destroy(h)
//
// The engine is host code over the library's own launchers (adp_conv_fwd, adp_maxpool2_fwd,
// adp_head_*_fwd, adp_prep_input, adp_tta_merge): the same kernels and schedule as nets.AdiposeV3Net.
// One handle per device and thread; calls are stream-ordered on the caller's stream (weights are
// uploaded synchronously by the first adp_forward after an adp_set_param).
#include <hip/hip_runtime.h>

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
};
struct HeadL {
  std::string name;
  int cin = 0, nout = 0, level = 0;
  std::vector<float> kernel, bias;
  float* W = nullptr;   // [nout][cin]
  float* b = nullptr;
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

  ~adp_handle() {
    for (auto& l : dense) { (void)hipFree(l.W); (void)hipFree(l.b); }
    for (auto& h : heads) { (void)hipFree(h.W); (void)hipFree(h.b); }
    for (auto& kv : buf) (void)hipFree(kv.second);
    (void)hipFree(wstage);
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
    dirty = false;
    return 0;
  }

  int conv(const char* name, int N, const void* srcA, int Hs, const void* srcB, void* out, float* accum,
           hipStream_t s) {
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
    return adp_conv_fwd(cfg.dtype, &d, &io, s);
  }

  // nets.AdiposeV3Net.forward (inference): x (N, S, S, 8) -> main probability map p_main (N, S, S)
  int forward(int N, hipStream_t s) {
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
    const size_t nsum = (size_t)N * sz[3] * sz[3] * ch[3];
    CL(adp_fill_f32(nsum, 0.f, b<float>("dsum_f"), s));
    const char* dl[6] = {"dl1", "dl2", "dl3", "dl4", "dl5", "dl6"};
    const char* dn[6] = {"dilate1", "dilate2", "dilate3", "dilate4", "dilate5", "dilate6"};
    for (int i = 0; i < 6; ++i)
      CL(conv(dn[i], N, i ? b(dl[i - 1]) : b("p3"), sz[3], nullptr, b(dl[i]), b<float>("dsum_f"), s));
    void* dsum = b("dsum_f");
    if (dt != ADP_DTYPE_F32) {
      CL(adp_cast(ADP_DTYPE_F32, dt, nsum, b("dsum_f"), b("dsum"), s));
      dsum = b("dsum");
    }
    CL(conv("up3_conv1", N, dsum, sz[3], nullptr, b("u3a"), nullptr, s));
    CL(conv("up3_conv2", N, b("d3"), sz[2], b("u3a"), b("u3b"), nullptr, s));
    CL(conv("up3_conv3", N, b("u3b"), sz[2], nullptr, b("u3"), nullptr, s));
    CL(conv("up2_conv1", N, b("u3"), sz[2], nullptr, b("u2a"), nullptr, s));
    CL(conv("up2_conv2", N, b("d2"), sz[1], b("u2a"), b("u2b"), nullptr, s));
    CL(conv("up2_conv3", N, b("u2b"), sz[1], nullptr, b("u2"), nullptr, s));
    CL(conv("up1_conv1", N, b("u2"), sz[1], nullptr, b("u1a"), nullptr, s));
    CL(conv("up1_conv2", N, b("d1"), sz[0], b("u1a"), b("u1b"), nullptr, s));
    CL(conv("up1_conv3", N, b("u1b"), sz[0], nullptr, b("u1"), nullptr, s));
    const HeadL& h = heads[head_idx.at("output_softmax")];
    return adp_head_softmax2_fwd(dt, (size_t)N * S * S, ch[0], h.cin, b("u1"), h.W, h.b, nullptr, nullptr,
                                 b<float>("p_main"), s);
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
  if (cfg->dtype == ADP_DTYPE_BF16) {   // inference channel layout of predictor.INFER_CPAD: 48/88/192/384
    const int cp[4] = {8, 8, 64, 64};
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
  if (!rc) rc = h->alloc("dsum_f", B * h->sz[3] * h->sz[3] * h->ch[3] * 4);
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
  std::memcpy(v->data(), host, n * sizeof(float));
  h->dirty = true;
  return 0;
}

extern "C" int adp_get_param(adp_handle* h, const char* layer, int slot, float* host, size_t n) {
  std::vector<float>* v = param_ref(h, layer, slot);
  if (!v || !host || n != v->size()) { adp::set_error("adp_get_param: unknown parameter or size mismatch"); return -1; }
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
