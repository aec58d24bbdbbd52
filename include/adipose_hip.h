/*
 * libadipose_hip — C ABI of the MI355X-native adipose U-Net hot path (gfx950 / CDNA4).
 *
 * The reference (MAGIC-SCAN/adipose_tissue-unet, TF 2.13 / Keras 2.13) has no FFI: its hot path is
 * the Keras graph built by AdiposeUNetV3.build_model (Segmentation/train_adipose_unet_v3.py:660-758)
 * plus the loss callables (:217-363), executed by TF/cuDNN. Each entry point below replaces one of
 * those implicit TF ops; the reference line it stands in for is cited on each declaration.
 *
 * Conventions
 *   - Every call returns 0 on success, <0 on error; adp_last_error() returns a thread-local message.
 *   - Pointers are DEVICE pointers unless stated; the caller owns every buffer.
 *   - Calls are asynchronous on the given hipStream_t (passed as void* so the header needs no HIP
 *     include) and never allocate, free or synchronise (safe to capture in a hipGraph).
 *   - dtype: ADP_DTYPE_F32 (parity path, exact f32 MFMA) or ADP_DTYPE_BF16 (throughput path,
 *     f32 accumulation); ADP_DTYPE_FP8 (e4m3fn operands, block-scaled MFMA, f32 accumulation) for
 *     forward-only launches (BASELINE.json configs[4]). Activations are NHWC with channel stride a
 *     multiple of 8.
 *   - GEMM weights are packed [Npad][Kpad] (output-channel major, K = taps*Cin_stride contiguous,
 *     Kpad = round_up(K,32), Npad = round_up(N,64)); tap order is row-major over (ky,kx).
 */
#ifndef ADIPOSE_HIP_H
#define ADIPOSE_HIP_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define ADP_DTYPE_F32 0
#define ADP_DTYPE_BF16 1
#define ADP_DTYPE_FP8 2 /* OCP e4m3fn, inference (forward) launches only */
#define ADP_ABI_VERSION 21 /* v4: adp_threshold_hist; v5: adp_maxpool2_bwd_bnr; v6: adp_aug_*, adp_percentile_normalize;
                              v7: handle engine adp_create / adp_forward / adp_*_param / adp_destroy;
                              v8: adp_train_step / adp_set_comm / adp_comm_*, adp_auc_metrics, adp_distance_transform, adp_boundary_metrics, adp_pack_weights_batch,
                              adp_bn_apply_maxpool2, adp_head_sigmoid_bwd_bnr;
                              v9: adp_conv_desc.bn_defer_fold + adp_bn_finalize_fold;
                              v10: adp_bn_bwd_apply_head, adp_head_sigmoid_bwd_bnr with dx = NULL, adp_conv_wgrad_bn;
                              v11: adp_sum_bf16; v12: adp_timing / adp_timing_read, unet_bn handle preset;
                              v13: adp_vec_mul (eval BatchNorm folded into the fp8 dequantisation scale);
                              v14: adp_scale_rows (eval BatchNorm folded into bf16 / f32 forward weights);
                              v15: adp_conv_wgrad_bn with dY = NULL (dz not stored), input-layer fused form;
                              v16: adp_bn_fold_reset, adp_debug_grad_flat;
                              v17: adp_wgrad_defer / adp_wgrad_flush
                              v18: adp_conv_io.act_outA;
                              v19: adp_conv_desc.CA_real / CB_real / Nout_real (zero-weight hints);
                              v20: adp_wgrad_release / adp_wgrad_arena_chunks (deferral arenas per (device, stream)), adp_get_option;
                              v21: adp_timing_filter */

typedef void* adp_stream_t; /* hipStream_t */

/* Geometry + epilogue of one implicit-GEMM convolution launch. */
typedef struct adp_conv_desc {
  int N, Hs, Ws;            /* source tensor(s) batch and spatial dims */
  int CA_stride, CB_stride; /* channel strides of source A / B (B = concat partner, 0 if none) */
  int upsample;             /* 1: nearest x2 upsample folded into the gather (UpSampling2D) */
  int Ho, Wo, stride;       /* output grid; input coord = o*stride + tap*dil - pad */
  int kh, kw, dil, pad;     /* tap grid */
  int Nout;                 /* GEMM N: output channels (padded) or 4*C for ConvTranspose */
  int relu;                 /* ReLU in the epilogue */
  float dropout_rate;       /* >0: inverted dropout after ReLU, stateless hash mask */
  unsigned dropout_seed;
  int out_stride;           /* channel stride of out */
  int out_mode;             /* 0 plain, 1 pixel-shuffle 2x2 (ConvTranspose), 2 channel split */
  int shuffle_c;            /* out_mode 1: channels per sub-pixel */
  int out2_stride, split_c; /* out_mode 2: channels >= split_c go to out2 */
  int mask_stride;          /* out = (acc [+addend]) * (mask>0) * mask_scale */
  float mask_scale;
  int mask2_stride;         /* same for the out2 part of a split store */
  float mask2_scale;
  int accum_stride;         /* accum (f32) += stored value */
  int bnr_stride;           /* channel stride of io->bnr_z */
  int out_fp8;              /* ADP_DTYPE_FP8 launches: 1 stores the output as fp8 e4m3 (else bf16); ADP_BF16
                               launches: 1 on an input layer (one 8-channel source, Nout 64) stores fp8 */
  int bn_defer_fold;        /* 1: leave this launch's BatchNorm statistics in the library's accumulator
                               replicas instead of adding them into io->bn_sum / bn_sqsum; the next launch
                               on the stream must be adp_bn_finalize_fold for those two vectors */
  int CA_real, CB_real;     /* v19, optional (0 = unknown): real channels of source A / B when the weight
                               columns of the pad channels [real, stride) are zeros (packed layers) */
  int Nout_real;            /* v19, optional (0 = unknown): real GEMM columns when weight rows [real, Nout)
                               are zeros. With these hints a kernel may skip products with zero weights
                               (f32 44-channel layers in 64-channel strides); results are unchanged */
} adp_conv_desc;

typedef struct adp_conv_io {
  const void* srcA;
  const void* srcB;
  const float* bn_scaleA; /* optional BatchNorm-apply + ReLU on load: x' = max(x*scale+shift, 0) */
  const float* bn_shiftA;
  const float* bn_scaleB;
  const float* bn_shiftB;
  const void* W;     /* packed weights, dtype of the launch */
  const float* bias; /* [Nout] or NULL */
  void* out;
  void* out2;
  const void* addend;
  const void* mask;
  const void* mask2;
  float* accum;
  float* bn_sum;     /* per-channel sum / sum of squares of the output (atomics), or NULL */
  float* bn_sqsum;
  /* optional fused BatchNorm-backward reduction over the stored output dA (out_mode 0; the
     adp_bn_bwd_reduce of the layer whose activation relu(z*scale+shift) this output is the
     gradient of): dbeta[c] += sum db, dgamma[c] += sum db*(z-mean)*invstd, db = dA*(z*scale+shift>0) */
  const void* bnr_z;
  const float* bnr_scale;
  const float* bnr_shift;
  const float* bnr_mean;
  const float* bnr_invstd;
  float* bnr_dgamma;
  float* bnr_dbeta;
  /* ADP_DTYPE_FP8 launches: per-GEMM-column dequantisation scale of W (adp_pack_weights_fp8) */
  const float* w_scale;
  /* (v18) with bn_scaleA / bn_shiftA on a one-source adp_conv_fwd: relu(srcA*scale+shift) is also stored here
     (srcA's shape and layout), bit-identical to adp_bn_apply(srcA) -> act_outA followed by the launch on
     act_outA; the persistent halo forward (3x3, 64 / 128 channels, BatchNorm statistics) does both in one
     launch, every other geometry runs exactly that pair */
  void* act_outA;
} adp_conv_io;

/* ---- library ---------------------------------------------------------------------------- */
const char* adp_last_error(void);
/* Name of the kernel instantiation the calling thread's last adp_conv_fwd / adp_conv_wgrad launched
   (as rocprofv3 prints it), for per-kernel timing and roofline accounting. */
const char* adp_last_kernel(void);
int adp_abi_version(void);
/* Build record: sha256 (hex) of the library's sources, in the Makefile's HASHED order (a caller can check that
 * a prebuilt binary matches the sources it ships with). */
const char* adp_source_hash(void);
/* Runtime switches, process-global (A/B of kernel variants in one process). value == INT_MIN restores
 * the built-in default. Kernel selection: "conv_fast" (2 = LDS-DMA kernels, default; 1 = register-staged;
 * 0 = generic), "fwd_tap64" / "wgrad_tap64" (0 off, 1 auto, 2+c force tile configuration c),
 * "tap64_bal", "tap64_korder", "wgrad_ra", "wgrad_blocks", "wgrad_min_chunk", "wgrad_glds_tn64";
 * epilogue store width (round 3, bit-identical either way): "tap64p_wide" (1), "tap64p_wide_f8" (0), "halop_wide"
 * (0 off, 1 tile-serial forms, 2 all, 3 default: all but the pipelined statistics forms), "cin8_wide" (1);
 * "wgrad_cin8_bna" (1: the input layer's fused BN-backward weight gradient when dY = NULL), "tap64_kpipe" (0:
 * mid-step barrier in the tap64 K loop); "wgrad_debug" / "fwd_debug" are timing-only ablations (results invalid). */
int adp_set_option(const char* name, int value);
/* The value adp_set_option gave `name`, INT_MIN when unset (v20; "tap64_ksplit_last" reports the split-K factor of the
 * last tap64 launch: 0 = none). */
int adp_get_option(const char* name);
/* Per-launch timing of the conv kernels (bench roofline; no reference counterpart). mode 1: clear the record
 * and start recording a HIP event pair around the MAIN kernel of every adp_conv_fwd / adp_conv_wgrad(_bn)
 * launch (the kernel adp_last_kernel names; statistic folds, split reduces, bias sums and BatchNorm applies
 * around it are excluded, so each pair times exactly one kernel of rocprofv3's list); 0: stop recording (the
 * record is kept); 2: stop and clear. */
int adp_timing(int mode);
/* Restricts the recording to launches whose kernel name (adp_last_kernel) equals `name` (NULL or "": every
 * launch): the bench times only its dominant kernel inside the timed region, where each event pair costs the
 * step time. */
int adp_timing_filter(const char* name);
/* Reads the record (synchronises on its events): *n = number of timed launches; for i < max: names[i *
 * name_len] = kernel name, ms[i] = its duration (-1 if its end was not marked). max = 0 only counts. */
int adp_timing_read(int max, char* names, int name_len, float* ms, int* n);

/* ---- dense layers (replace Conv2D / Conv2DBackpropInput / Conv2DBackpropFilter / BiasAdd /
 *      Relu / ResizeNearestNeighbor / ConcatV2 / AddN / Dropout of
 *      Segmentation/train_adipose_unet_v3.py:668-710, and ConvTranspose2D of the unet_bn preset) */
int adp_conv_fwd(int dtype, const adp_conv_desc* d, const adp_conv_io* io, adp_stream_t s);
/* ADP_DTYPE_FP8: srcA/srcB/W fp8 e4m3, channel strides and K multiples of 128 (one 128-channel K step
 * per tap), acc[m][n] * w_scale[n] (+ bias, ReLU) stored as bf16 or fp8 (desc.out_fp8); out_mode 0 or 1;
 * no BatchNorm / addend / mask / accumulate / dropout epilogue terms. */
/* dW[Npad][Kpad] (+)= sum_m dY[m][n] * X_tap(k)[m]; dB[n] (+)= sum_m dY[m][n]. f32 accumulators,
 * caller zeroes them. The gather is described by d/io exactly as for the forward launch. */
int adp_conv_wgrad(int dtype, const adp_conv_desc* d, const adp_conv_io* io, const void* dY,
                   int dy_stride, float* dW, float* dB, adp_stream_t s);
/* The BatchNorm backward of the layer this conv feeds (adp_bn_bwd_apply's arguments): dY of the weight
 * gradient is dz = bn_bwd_apply(dA, z) (dgamma / dbeta already reduced). */
typedef struct adp_bn_bwd_args {
  const void* dA;      /* gradient wrt relu(z*scale + shift), [M][dy_stride] */
  const void* z;       /* the layer's pre-BatchNorm output, [M][dy_stride] */
  const float *scale, *shift, *mean, *invstd, *gamma, *dgamma, *dbeta;
  float count;
} adp_bn_bwd_args;
/* adp_bn_bwd_apply(bn -> dY) followed by adp_conv_wgrad(dY), as one launch where the persistent halo
 * weight-gradient kernel takes the shape (3x3 stride-1 layers with <= 2 64-channel input chunks): dz is
 * computed while the weight gradient loads its tiles and stored into dY (for the data-gradient launch),
 * bit-identical to the two-launch form, which runs otherwise. dY may be NULL when dB is NULL and nothing
 * reads dz (the input layer has no data gradient): the fused forms then store nothing -- and the
 * input-layer kernel (one 8-channel source, 64 outputs) takes the fused form too -- while the two-launch
 * form computes dz in library scratch. */
int adp_conv_wgrad_bn(int dtype, const adp_conv_desc* d, const adp_conv_io* io, const adp_bn_bwd_args* bn,
                      void* dY, int dy_stride, float* dW, float* dB, adp_stream_t s);

/* Repack f32 master weights into the launch layout: mode 0 = cast only (forward);
 * mode 1 = 3x3 flip+transpose (data-gradient of a conv), mode 2 = ConvTranspose transpose. */
int adp_pack_weights(int dtype_out, int mode, int taps, int Cin_s, int Nout, const float* src,
                     int src_kpad, void* dst, int dst_rows, int dst_kpad, adp_stream_t s);
/* Modes 1/2 of adp_pack_weights for up to ADP_PACK_MAX_JOBS layers in one launch (LDS-tiled transpose,
 * coalesced both ways): dst[ci][t*Nout + co] = src[co][(taps-1-t)*Cin_s + ci], zeros elsewhere. */
#define ADP_PACK_MAX_JOBS 24
typedef struct adp_pack_job {
  const float* src;
  void* dst;
  int taps, Cin_s, Nout, src_kpad, dst_rows, dst_kpad;
} adp_pack_job;
int adp_pack_weights_batch(int dtype_out, int n, const adp_pack_job* jobs, adp_stream_t s);
/* Forward-layout fp8 weights with a per-row (output channel) scale: scale[r] = max_k |src[r][k]| / 448
 * (1 for an all-zero row), dst[r][k] = e4m3(src[r][k] / scale[r]) (saturating, round to nearest even). */
int adp_pack_weights_fp8(int rows, const float* src, int src_kpad, void* dst, int dst_kpad, float* scale,
                         adp_stream_t s);

/* ---- pooling / upsampling (MaxPooling2D :670,674,678; UpSampling2D grad) ------------------- */
int adp_maxpool2_fwd(int dtype, int N, int H, int W, int C_stride, const void* src,
                     const float* bn_scale, const float* bn_shift, void* dst, adp_stream_t s);
/* 2x2 max-pool with an fp8 e4m3 output; src of dtype dtype_in (F32, BF16 or FP8) */
int adp_maxpool2_fwd_fp8(int dtype_in, int N, int H, int W, int C_stride, const void* src, void* dst_fp8,
                         adp_stream_t s);
int adp_maxpool2_bwd(int dtype, int N, int H, int W, int C_stride, const void* src,
                     const float* bn_scale, const float* bn_shift, const void* dpool,
                     const void* addend, const void* mask, float mask_scale, void* dsrc,
                     adp_stream_t s);
/* unet_bn encoder pool backward: dsrc = route_argmax(dpool) + addend (no BN-on-load, no mask), with the
 * BatchNorm-backward reduction of the layer whose activation src = relu(z*scale+shift) fused in:
 * dbeta += sum db, dgamma += sum db*(z-mean)*invstd, db = dsrc*(z*scale+shift > 0) over the stored dsrc
 * (replaces adp_maxpool2_bwd + adp_bn_bwd_reduce; train_adipose_unet_v3.py:670 MaxPooling2D grad).
 * src may be NULL: the argmax then runs over relu(z*scale+shift) recomputed and rounded to dtype, the
 * values adp_bn_apply / adp_bn_apply_maxpool2 store (one full-resolution read less) */
int adp_maxpool2_bwd_bnr(int dtype, int N, int H, int W, int C_stride, const void* src, const void* dpool,
                         const void* addend, void* dsrc, const void* z, const float* scale, const float* shift,
                         const float* mean, const float* invstd, float* dgamma, float* dbeta, adp_stream_t s);
/* unet_bn encoder: act = relu(z * scale + shift) (adp_bn_apply) and pool = maxpool2(act) in one pass */
int adp_bn_apply_maxpool2(int dtype, int N, int H, int W, int C_stride, const void* z, const float* scale,
                          const float* shift, void* act, void* pool, adp_stream_t s);
int adp_upsample2_bwd(int dtype, int N, int Hs, int Ws, int C_stride, const void* dup,
                      const void* addend, const void* mask, float mask_scale, void* dsrc,
                      adp_stream_t s);
/* out = (a [+ b]) * (mask>0 ? mask_scale : 0) [mask optional]; elementwise over n elements */
int adp_ew_add_mask(int dtype, size_t n, const void* a, const void* b, const void* mask,
                    float mask_scale, void* out, adp_stream_t s);
int adp_cast(int dtype_in, int dtype_out, size_t n, const void* src, void* dst, adp_stream_t s);
int adp_fill_f32(size_t n, float value, float* dst, adp_stream_t s);
/* out = bf16(sum of nsrc (1..8) bf16 maps of n elements, f32 sum in source order): the dilated
   bottleneck's Add (train_adipose_unet_v3.py:688) as one pass after its six convs; n % 8 == 0, srcs is a
   host array of 16-B aligned device pointers */
int adp_sum_bf16(int nsrc, const void* const* srcs, size_t n, void* out, adp_stream_t s);

/* ---- BatchNorm (unet_bn preset; training-mode batch statistics) -------------------------- */
int adp_bn_finalize(int C, float count, const float* sum, const float* sqsum, const float* gamma,
                    const float* beta, float eps, float momentum, float* scale, float* shift,
                    float* mean, float* invstd, float* running_mean, float* running_var,
                    adp_stream_t s);
/* adp_bn_finalize of statistics a conv launch left in the accumulator replicas (bn_defer_fold): first
 * sum[c] += replicas, sqsum[c] += replicas (the replicas are re-zeroed), then the finalize; one launch in
 * place of the fold + finalize pair. */
int adp_bn_finalize_fold(int C, float count, float* sum, float* sqsum, const float* gamma, const float* beta,
                         float eps, float momentum, float* scale, float* shift, float* mean, float* invstd,
                         float* running_mean, float* running_var, adp_stream_t s);
/* Drops a bn_defer_fold record that never reached its adp_bn_finalize_fold (an error or exception between the
 * two) and re-zeroes the replicas, stream-ordered on s; a no-op when nothing is pending, and when the pending
 * record was made on another stream (another caller's fold, possibly still in flight). Trainer steps and
 * adp_train_step call it first, so a failed step cannot poison the replicas for the rest of the process. */
int adp_bn_fold_reset(adp_stream_t s);
/* Deferred weight-gradient reductions (round 5). The weight / bias gradient launches (adp_conv_wgrad, _bn) sum per-block
 * partial slabs in a fixed order (deterministic) with a small reduce launch each. Between adp_wgrad_defer(1, s) and
 * adp_wgrad_flush(s), launches on stream s write their slabs to a per-stream arena and only record the reduction;
 * adp_wgrad_flush launches every recorded reduction as one kernel (same arithmetic: bit-identical gradients) and ends
 * the deferral. Until the flush the dW / dB buffers of those launches are NOT final: call it before anything reads
 * them (the optimizer, a gradient all-reduce). adp_wgrad_defer(0, s) with reductions pending is an error. */
int adp_wgrad_defer(int on, adp_stream_t s);
int adp_wgrad_flush(adp_stream_t s);
/* The deferral arena of (current device, stream s) -- chunks of >= 256 MiB allocated by the first deferred steps and reused
 * afterwards -- freed, and the stream forgotten (v20). Synchronises s; an error with reductions pending. Call it before
 * destroying a stream that deferred. adp_wgrad_arena_chunks: the number of arena chunks of (device, s) (test hook). */
int adp_wgrad_release(adp_stream_t s);
int adp_wgrad_arena_chunks(adp_stream_t s);
/* a = relu(z*scale + shift), the post-BatchNorm activation, materialised once per layer */
int adp_bn_apply(int dtype, size_t M, int C, const void* z, const float* scale, const float* shift,
                 void* out, adp_stream_t s);
/* the same activation stored as fp8 e4m3 (z of dtype dtype_in): the operand of an fp8 conv launch */
int adp_bn_apply_fp8(int dtype_in, size_t M, int C, const void* z, const float* scale, const float* shift,
                     void* out_fp8, adp_stream_t s);
/* out[i] = a[i] * b[i] (f32 vectors): e.g. an fp8 layer's per-column dequantisation scale times its eval
   BatchNorm scale, so that the conv epilogue writes relu(bn(z)) directly (UNetBN.forward_fp8) */
int adp_vec_mul(size_t n, const float* a, const float* b, float* out, adp_stream_t s);
/* dst[r][c] = src[r][c] * scale[r] (0 for r >= nscale), c < cols, stored as dtype_out (ADP_DTYPE_F32 / BF16): a
   layer's forward weights ([Npad][Kpad] master layout) with its eval BatchNorm scale folded in, so that the conv
   epilogue (bias = BN shift, ReLU) writes relu(bn(z)) directly (UNetBN.forward(train=False)) */
int adp_scale_rows(int dtype_out, int rows, int cols, const float* src, int src_ld, const float* scale, int nscale,
                   void* dst, int dst_ld, adp_stream_t s);
/* dBN = dA * (relu(z*scale+shift) > 0); dgamma += sum dBN*xhat; dbeta += sum dBN */
int adp_bn_bwd_reduce(int dtype, size_t M, int C, const void* dA, const void* z, const float* scale,
                      const float* shift, const float* mean, const float* invstd, float* dgamma,
                      float* dbeta, adp_stream_t s);
int adp_bn_bwd_apply(int dtype, size_t M, int C, const void* dA, const void* z, const float* scale,
                     const float* shift, const float* mean, const float* invstd,
                     const float* gamma, const float* dgamma, const float* dbeta, float count,
                     void* dz, adp_stream_t s);
/* adp_bn_bwd_apply of the layer under the unet_bn sigmoid head with dA recomputed instead of read:
 * dA[m][c] = dtype(dp[m] * p[m] * (1 - p[m]) * W[c]) (0 for c >= Cin; Cin % 8 == 0, W 16-B aligned), the value adp_head_sigmoid_bwd_bnr
 * stores, so that launch can run with dx = NULL (one full-resolution write and read fewer; bit-identical dz) */
int adp_bn_bwd_apply_head(int dtype, size_t M, int C, int Cin, const float* W, const float* p, const float* dp,
                          const void* z, const float* scale, const float* shift, const float* mean,
                          const float* invstd, const float* gamma, const float* dgamma, const float* dbeta,
                          float count, void* dz, adp_stream_t s);

/* ---- heads (Conv2D(2,1,softmax)[...,1] :729-731; Conv2D(1,1,sigmoid) :715,722) ------------- */
/* p = softmax(W x + b)[1] = sigmoid(z1 - z0); W f32 [2][Cin], b f32 [2] */
int adp_head_softmax2_fwd(int dtype, size_t M, int C_stride, int Cin, const void* x, const float* W,
                          const float* b, const float* bn_scale, const float* bn_shift, float* p,
                          adp_stream_t s);
int adp_head_softmax2_bwd(int dtype, size_t M, int C_stride, int Cin, const void* x, const float* W,
                          const float* bn_scale, const float* bn_shift, const float* p,
                          const float* dp, const void* addend, const void* mask, float mask_scale,
                          void* dx, float* dW, float* db, adp_stream_t s);
/* p = sigmoid(W x + b); W f32 [Cin], b f32 [1] */
int adp_head_sigmoid_fwd(int dtype, size_t M, int C_stride, int Cin, const void* x, const float* W,
                         const float* b, const float* bn_scale, const float* bn_shift, float* p,
                         adp_stream_t s);
int adp_head_sigmoid_bwd(int dtype, size_t M, int C_stride, int Cin, const void* x, const float* W,
                         const float* bn_scale, const float* bn_shift, const float* p,
                         const float* dp, const void* addend, const void* mask, float mask_scale,
                         void* dx, float* dW, float* db, adp_stream_t s);
/* unet_bn head backward with the BatchNorm-backward reduction of the layer under it fused (adp_bn_bwd_reduce):
 * z = that layer's pre-BN output (the head reads relu(z*sc+sh)), dx = dL/d relu(bn(z)) stored, and
 * dbeta += sum db, dgamma += sum db*(z-mean)*invstd with db = dx*(z*sc+sh > 0) over the (rounded) dx;
 * dx may be NULL (the sums are the same; adp_bn_bwd_apply_head then recomputes dx) */
int adp_head_sigmoid_bwd_bnr(int dtype, size_t M, int C_stride, int Cin, const void* z, const float* W,
                             const float* scale, const float* shift, const float* mean, const float* invstd,
                             const float* p, const float* dp, void* dx, float* dW, float* db, float* dgamma,
                             float* dbeta, adp_stream_t s);
/* tf.image.resize(..., method='bilinear') (half-pixel centres, no antialias), 1 channel, f32
 * (:716-719, :723-726) and its adjoint. */
int adp_resize_bilinear_fwd(int N, int Hs, int Ws, int Ho, int Wo, const float* src, float* dst,
                            adp_stream_t s);
int adp_resize_bilinear_bwd(int N, int Hs, int Ws, int Ho, int Wo, const float* dout, float* dsrc,
                            adp_stream_t s);

/* ---- losses & metrics (dice_loss / combined_loss_* / OHEM :217-363; dice_coef model.py:93-98) */
/* stats[0..7] += {sum y*p', sum y, sum p', sum y*p, sum y, sum p (raw y, p), #((p>0.5)==y),
 *                 sum y*(p>0.5)} where
 * p' = clip(p,1e-7,1-1e-7) and y is the (optionally smoothed) label; row_bce[b*H+h] = mean_w BCE. */
int adp_loss_rows(int N, int H, int W, const float* p, const float* y, int smooth, float eps_pos,
                  float eps_neg, float* row_bce, double* stats, adp_stream_t s);
/* One block per image: selects rows (OHEM top-k with k = int(H*keep_ratio) or all rows), writes
 * row_coef[b*H+h] = weight/(norm_rows*W) for selected rows else 0, and out[0] += weight*bce_part,
 * with norm_rows the GLOBAL number of selected rows (all ranks). */
int adp_loss_select(int N, int H, int W, const float* row_bce, int ohem, float keep_ratio,
                    float weight, float norm_rows, float* row_coef, double* out, adp_stream_t s);
/* dp (+)= row_coef*dBCE/dp + weight*dDice/dp (through the clip), given GLOBAL dice stats. */
int adp_loss_grad(int N, int H, int W, const float* p, const float* y, int smooth, float eps_pos,
                  float eps_neg, const float* row_coef, const double* stats, float weight,
                  int accumulate, float* dp, adp_stream_t s);
/* tp, fp, fn, tn of (pred>thr) vs (true>0.5) (full_evaluation_enhanced.py:721-785), int64 out */
int adp_pixel_counts(size_t n, const float* pred, const float* truth, float thr,
                     unsigned long long* counts, adp_stream_t s);
/* Threshold sweep of optimize_threshold_f1(_slide_level) (full_evaluation_enhanced.py:891-980) in one pass:
 * thr = nthr (<= 64) ascending HOST doubles; hist[b*(nthr+1) + j] (+)= #pixels with truth bit b
 * (truth > 0.5) and j = #{t : pred > thr[t]}. tp(t) = sum_{j>t} hist[nthr+1+j], fp(t) = sum_{j>t} hist[j]. */
int adp_threshold_hist(size_t n, const float* pred, const float* truth, int nthr, const double* thr,
                       unsigned long long* hist, adp_stream_t s);

/* ---- the rest of the src/utils/model.py loss / metric surface (not on the v3 training step) ---------- */
/* weighted_dice_loss / weighted_bce_dice_loss weight map (model.py:104-116, 140-151): y (B,H,W) f32 is expanded
 * to (1,B,H,W) channels_last, so K.pool2d(ksize x ksize, stride 1, 'same', 'avg') averages over (B, H) per W
 * (TF 'SAME' average: padding excluded from the count); weight = 1 + 2 * (0.005 < avg < 0.995); wsum[0] +=
 * sum(weight) (f64, caller zeroes). tmp: B*H*W f32 scratch. ksize odd (21 in the reference). */
int adp_border_weight(int B, int H, int W, int ksize, const float* y, float* tmp, float* weight, double* wsum,
                      adp_stream_t s);
/* With w = weight * (n / wsum[0]) (f32, the w0/w1 renormalisation): stats[0..4] += {sum w^2 y p, sum w^2 y,
 * sum w^2 p, sum bce_w, sum w}, bce_w = (1-y) l + (1 + (w-1) y)(log(1 + exp(-|l|)) + max(-l, 0)),
 * l = log(p'/(1-p')), p' = clip(p, 1e-7, 1-1e-7) (weighted_dice_coeff :120-125, weighted_bce_loss :127-136). */
int adp_weighted_loss_stats(size_t n, const float* y, const float* p, const float* weight, const double* wsum,
                            double* stats, adp_stream_t s);
/* dp = wbce * d(stats[3]/stats[4])/dp + wdice * d(1 - (2 stats[0] + 1)/(stats[1] + stats[2] + 1))/dp (TF's
 * subgradients of clip / abs / maximum), from the final stats. */
int adp_weighted_loss_grad(size_t n, const float* y, const float* p, const float* weight, const double* wsum,
                           const double* stats, float wbce, float wdice, float* dp, adp_stream_t s);
/* K.mean / K.min / K.max / K.std (population) of n floats (act_mean, act_min, act_max, act_std, mean_diff
 * model.py:21-34): out (device f64[4]) = {mean, min, max, std}; work >= 1024 * 40 bytes. */
int adp_value_stats(size_t n, const float* x, void* work, double* out, adp_stream_t s);
/* argmax / argmin over the last axis (first occurrence) of y and p, rows x W (model.py:36-91): out (int64[7],
 * caller zeroes) += {tru_pos = sum at*ap, fls_pos = sum clip(ap-at,0,1), tru_neg = sum it*ip,
 * fls_neg = sum clip(ip-it,0,1), #(at*ap >= 1), #(ap >= 1), #(at >= 1)} (the last three: precision_onehot /
 * recall_onehot's rounded counts). */
int adp_onehot_counts(int rows, int W, const float* y, const float* p, unsigned long long* out, adp_stream_t s);

/* ---- training-time augmentation + normalisation of gray (H, W) f32 planes (src/utils/data.py:13-264,
 * 398-429); random parameters are drawn by the host in the reference's RandomState order ---------- */
/* np.rot90(k) then fliplr then flipud (random_rotation_90 / random_flip, data.py:13-29); out of place */
int adp_aug_geom(int H, int W, const float* src, float* dst, int k, int flip_lr, int flip_ud, adp_stream_t s);
/* mode 0 brightness clip(x*f,0,255), 1 contrast clip((x-m)*f+m,0,255), 2 gamma (x/255)^f*255 (:32-50),
 * 3 z-score (x-m)/f (TileDataset, train_adipose_unet_v3.py:589-590) */
int adp_aug_photometric(size_t n, const float* src, float* dst, int mode, float f, float m, adp_stream_t s);
/* clip(x + noise, 0, 255) with noise f64 (random_gaussian_noise, :63-69) */
int adp_aug_noise(size_t n, const float* src, const double* noise, float* dst, adp_stream_t s);
/* *out += sum(src) in f64 (contrast's image.mean()) */
int adp_aug_sum(size_t n, const float* src, double* out, adp_stream_t s);
/* separable Gaussian (cv2.GaussianBlur, BORDER_REFLECT_101), taps[2r+1]; dtype64: src/tmp/dst are f64 */
int adp_aug_blur(int dtype64, int H, int W, const void* src, void* tmp, void* dst, const float* taps, int radius,
                 adp_stream_t s);
/* random_scale (:72-106): cv2.resize to (Hn, Wn) (linear, or nearest for masks) + center crop / pad */
int adp_aug_scale(int H, int W, int Hn, int Wn, const float* src, float* dst, int nearest, adp_stream_t s);
/* elastic_transform (:109-145): remap image (linear, reflect) and mask (nearest, 0) by (x+dx*alpha, y+dy*alpha) */
int adp_aug_remap(int H, int W, const float* src, const float* msrc, const double* dx, const double* dy, double alpha,
                  float* dst, float* mdst, adp_stream_t s);
/* normalize_image(method='percentile') (:398-429) with exact order statistics (radix select on the
 * device); work >= 64 + 32768 bytes; p_out (nullable) receives (p_low, p_high) values */
int adp_percentile_normalize(size_t n, const float* src, float* dst, double p_low, double p_high, void* work,
                             float* p_out, adp_stream_t s);

/* ---- optimizer (Keras Adam / AdamW, :800-806) --------------------------------------------- */
int adp_adam(size_t n, float* param, const float* grad, float* m, float* v, float lr, float beta1,
             float beta2, float eps, int step, float weight_decay, float grad_scale, adp_stream_t s);
int adp_ema(size_t n, float* ema, const float* param, float decay, adp_stream_t s);

/* ---- input / inference plumbing (predict_single :153-158, TTA :181-229, SW/blend
 *      full_evaluation_enhanced.py:115-329) ------------------------------------------------- */
/* dst[n, y, x, c] = (src_view(view)[n, y, x, c] - mean) / (std + 1e-10); src f32 rows of Cin
 * interleaved channels with a row stride of src_row_stride pixels and an image stride of
 * src_img_stride floats (<= 0: dense), so a sliding-window tile is read in place from the full
 * image; dst NHWC with C_stride >= Cin (pad channels zeroed); view 0..7 = TTA forward transform. */
int adp_prep_input(int dtype, int N, int H, int W, int Cin, const float* src,
                   long long src_row_stride, long long src_img_stride, float mean, float std,
                   int view, int C_stride, void* dst, adp_stream_t s);
/* out[y,x] = mean_v inverse_view(v)(probs[v])[y,x] over nviews views listed in views[] (host) */
int adp_tta_merge(int H, int W, int nviews, const int* views, const float* probs, float* out,
                  adp_stream_t s);
int adp_blend_accum(int H, int W, int T, int y0, int x0, const float* tile, const float* weight,
                    float* acc, float* wsum, adp_stream_t s);
int adp_blend_finalize(size_t n, const float* acc, const float* wsum, float floor_, float* out,
                       adp_stream_t s);

/* ROC AUC and average precision of a probability map against a mask (full_evaluation_enhanced.py:847-888:
 * roc_auc_score / average_precision_score on the flattened pixels, truth > 0.5 positive; ties grouped by
 * identical score). out: device f64[2] = {roc_auc, pr_auc}, NaN when only one class is present. */
int adp_auc_metrics(size_t n, const float* pred, const float* truth, double* out, adp_stream_t s);
/* scipy.ndimage.distance_transform_edt(~(src > thr), sampling=(sy, sx)): dist (device f64 H x W) = Euclidean
 * distance to the nearest pixel with src > thr (inf if there is none). Exact (separable lower envelope). */
int adp_distance_transform(int H, int W, const float* src, float thr, double sy, double sx, double* dist,
                           adp_stream_t s);
/* calculate_boundary_metrics (full_evaluation_enhanced.py:788-844) on the GPU: out (HOST f64[2]) =
 * {hausdorff95, assd}; 0 / 0 for two empty masks, inf for one empty mask or an empty surface. The
 * reference's pairing is kept (each distance map is sampled at its own mask's surface). Synchronises s. */
int adp_boundary_metrics(int H, int W, const float* pred, const float* truth, float thr, double sy, double sx,
                         double* out, adp_stream_t s);

/* BoundaryRefiner.refine (full_evaluation_enhanced.py:357-393) of one (H, W) f32 probability map: m = u8(mask*255),
 * ellipse (ksize; row_lo / row_hi = HOST arrays of ksize column extents, getStructuringElement(MORPH_ELLIPSE))
 * erode / dilate -> band = dilated>0 xor eroded>0, bilateral filter (d, sigma_color, sigma_space;
 * cv2.bilateralFilter semantics, BORDER_REFLECT_101) inside the band, MORPH_OPEN then MORPH_CLOSE, out = f32(x / 255).
 * work: >= 4*H*W bytes. ksize <= 31, d / 2 <= 15. */
int adp_boundary_refine(int H, int W, const float* mask, int ksize, const int* row_lo, const int* row_hi, int d,
                        float sigma_color, float sigma_space, void* work, float* out, adp_stream_t s);

/* ---- handle-level engine: native adipose_v3 inference for non-Python callers ---- */
#define ADP_PRESET_ADIPOSE_V3 0 /* AdiposeUNetV3.build_model (train_adipose_unet_v3.py:660-758) */
#define ADP_PRESET_UNET_BN 1    /* BASELINE.json configs 2/3/5: L levels, base width, [conv3x3 -> BatchNorm -> ReLU] x 2,
                                   MaxPool 2x2, ConvTranspose 2x2/s2 + skip concat, 1x1 sigmoid head (no reference
                                   code; the Python schedule is nets.UNetBN) */
typedef struct adp_handle adp_handle; /* opaque: topology, packed weights, activation buffers */
typedef struct adp_config {
  int preset;            /* ADP_PRESET_ADIPOSE_V3 or ADP_PRESET_UNET_BN */
  int tile;              /* S (the reference hard-codes 1024), multiple of 8 (unet_bn: of 2^(levels-1)) */
  int max_batch;         /* images x TTA views per forward (activation buffers are sized for it) */
  int dtype;             /* ADP_DTYPE_F32 (the reference's fp32 numerics) or ADP_DTYPE_BF16 */
  int deep_supervision;  /* adipose_v3: 1 = the aux_out1 / aux_out2 heads exist (checkpoint layout); inference = main_out */
  int init_nb;           /* adipose_v3 base width, 44 (build_model(init_nb=44)) */
  /* v12 */
  int levels;            /* unet_bn: resolution levels (0 -> 5; configs[2] = 5, configs[1] = 4) */
  int base;              /* unet_bn: level-0 width (0 -> 64) */
  int in_ch;             /* unet_bn: input channels (0 -> 3), tiles (S, S, in_ch) interleaved f32 */
  float dropout_rate;    /* adipose_v3: build_model(dropout_rate) (0.3), used by adp_train_step when its cfg's
                            dropout_rate < 0; unet_bn has no dropout layers (ignored) */
  unsigned seed;         /* dropout mask stream: step k uses hash seed (seed + k) * 7919 + 17 (0 = the Python
                            Trainer's stream) */
} adp_config;
int adp_create(const adp_config* cfg, int device, adp_handle** out);
int adp_destroy(adp_handle* h);
/* i-th parameterised layer name (Keras layer names), NULL past the end */
const char* adp_param_name(const adp_handle* h, int i);
/* adipose_v3: slot 0 = kernel (Keras HWIO for convs, (1,1,Cin,Nout) for heads), 1 = bias. unet_bn: conv layers
 * (enc*_conv*, dec*_conv*) 0 = kernel HWIO, 1 = gamma, 2 = beta, 3 = moving mean, 4 = moving variance;
 * ConvTranspose dec*_up 0 = kernel (Cin, Cout, 2, 2), 1 = bias; head 0 = kernel (1,1,Cin,1), 1 = bias.
 * n = element count. unet_bn parameter I/O is synchronous (the device is synchronised first). */
int adp_param_size(adp_handle* h, const char* layer, int slot, size_t* n);
int adp_set_param(adp_handle* h, const char* layer, int slot, const float* host, size_t n);
int adp_get_param(adp_handle* h, const char* layer, int slot, float* host, size_t n);
/* The gradient of a parameter slot from the last adp_train_step (after its all-reduce), same layout as
 * adp_get_param; synchronous. Errors before the first step and for the running-statistics slots. */
int adp_get_grad(adp_handle* h, const char* layer, int slot, float* host, size_t n);
/* Test hook of the bucketed all-reduce (v16): which = 0 copies the whole flat gradient buffer of the last
 * adp_train_step (n = its element count, adp_debug_grad_flat(h, 0, NULL, 0) -> error message names it);
 * which = 1 copies the snapshot taken on the communication stream as each bucket's all-reduce was issued,
 * recorded only while option "dp_snapshot" is 1. With a one-rank communicator (the in-place SUM changes
 * nothing) the two are equal iff no gradient was written after its bucket started. Synchronous. */
int adp_debug_grad_flat(adp_handle* h, int which, float* host, size_t n);
/* predict_single / TTA (segmentation_inference.py:153-229): images = n device f32 (S,S) raw gray tiles
 * img_stride floats apart (<= 0: dense); prob = n device f32 (S,S) main_out probabilities;
 * (x - mean)/(std + 1e-10) on load; tta_mode 0 none, 1 minimal (id, flipH), 2 basic (+flipV, rot90),
 * 3 full (8 views). Stream-ordered; the first call after adp_set_param uploads the weights
 * (synchronous). One handle per device and thread. */
int adp_forward(adp_handle* h, const float* images, int n, long long img_stride, float mean, float std,
                int tta_mode, float* prob, adp_stream_t s);

/* unet_bn: images are n device f32 (S, S, in_ch) interleaved tiles (img_stride floats apart, <= 0: dense);
 * BatchNorm uses the running statistics (eval). */
/* One training step of AdiposeUNetV3 (model.net.fit, train_adipose_unet_v3.py:1316-1324) on the handle:
 * forward with dropout -> main / deep-supervision losses and their gradients (compile_model :780-879:
 * OHEM or BCE+Dice main head, BCE+Dice aux heads, label smoothing :244-279, weights 1.0 / 0.4 / 0.3) ->
 * backward -> [SUM all-reduce of the gradients over the communicator of adp_set_comm] -> Adam / AdamW
 * (Keras 2.13 update, :800-806). Frozen encoder (freeze_encoder_layers :760-772): no encoder
 * gradients or updates. x: n device f32 (S,S) normalised images, y: n device f32 (S,S) labels in {0,1};
 * n <= max_batch. metrics (host, 6 floats, the call synchronises the stream): loss, main_out_loss,
 * aux_out1_loss, aux_out2_loss, main_out_dice_coef, main_out_binary_accuracy (Keras' per-batch values;
 * with a communicator: of the global batch). The first call allocates the optimizer state (m, v = 0).
 * With a communicator the gradients are SUM-all-reduced in ~16 MB buckets on a communication stream, each as
 * soon as the backward has produced all of its layers (overlapping the remaining backward launches).
 * unet_bn: x is n (S, S, in_ch) f32 normalised tiles; the loss is the main head's (OHEM or BCE + Dice per
 * use_hard_mining, label smoothing), BatchNorm uses batch statistics and updates the running ones
 * (momentum 0.1, eps 1e-5); freeze_encoder must be 0. */
typedef struct adp_train_cfg {
  int use_hard_mining;       /* OHEM main loss (--use-hard-mining, default on) */
  float hard_example_ratio;  /* 0.7 */
  int use_label_smoothing;
  float epsilon_pos, epsilon_neg;          /* 0.03, 0.07 */
  float w_main, w_aux1, w_aux2;            /* 1.0, 0.4, 0.3 */
  int optimizer;             /* 0 Adam, 1 AdamW (weight_decay) */
  float beta1, beta2, eps, weight_decay;   /* 0.9, 0.999, 1e-7, 0.01 */
  float dropout_rate;        /* 0.3 (build_model dropout_rate) */
  int freeze_encoder;        /* phase 1 */
} adp_train_cfg;
int adp_train_step(adp_handle* h, const float* x, const float* y, int n, const adp_train_cfg* cfg, float lr,
                   float* metrics, adp_stream_t s);
/* Data-parallel training: comm is an RCCL ncclComm_t (one rank per GPU); NULL detaches. RCCL is loaded
 * at run time (librccl.so.1). The helpers create a communicator without another framework:
 * adp_comm_unique_id fills 128 bytes on one rank, which every rank passes to adp_comm_init. */
int adp_set_comm(adp_handle* h, void* comm);
int adp_comm_unique_id(void* id128);
int adp_comm_init(int nranks, const void* id128, int rank, void** comm);
int adp_comm_destroy(void* comm);

#ifdef __cplusplus
}
#endif
#endif
