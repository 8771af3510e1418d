/*
 * dmx.h — C ABI of libdmx.so, the MI355X (gfx950) native CFG denoising loop.
 *
 * The reference (S-Taichiii/diffusion-model) is pure Python and has no FFI; its
 * drop-in boundary is the duck-typed Python surface:
 *   Diffuser.denoise_cond / sample_latent_cond   (reference diff.py:127-162, 174-369)
 *   UnetCondWithGeomHead.forward                  (reference models/unet_cond_geom.py:79-100)
 *   VAE.decode                                    (reference models/vae.py:64-69)
 * Those Python classes are re-implemented in diffusion-model_amd/ and call the
 * entry points below through ctypes (diffusion-model_amd/dmx/_lib.py).  Each entry
 * point cites the reference call it replaces.
 *
 * Conventions
 *   - every function returns 0 on success, a DMX_E* code otherwise; the message is
 *     available from dmx_last_error() (thread-local).  No C++ exception crosses
 *     this boundary.
 *   - tensors are caller-owned DEVICE pointers (contiguous, fp32 NCHW for x/eps/
 *     images, int64 for t/y, fp32 (n,12) for vals/mask); weights and workspace are
 *     owned by the dmx objects.
 *   - `stream` is a hipStream_t (void* here so that the header needs no HIP).
 *     All work is enqueued on it; calls on one model must be serialised by the
 *     caller.
 */
#ifndef DMX_H_
#define DMX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DMX_OK 0
#define DMX_E_ARG 1      /* invalid argument / shape (reference: ValueError / AssertionError) */
#define DMX_E_STATE 2    /* object not ready (e.g. weights missing) */
#define DMX_E_HIP 3      /* HIP runtime failure */
#define DMX_E_INTERNAL 4

/* model kinds */
#define DMX_UNET_COND_GEOM 1 /* models/unet_cond_geom.py:26 UnetCondWithGeomHead */
#define DMX_UNET_COND 2      /* models/unet_cond.py:102    UnetCond               */
#define DMX_UNET 3           /* models/unet.py:101          Unet (unconditional)  */
#define DMX_VAE 4            /* models/vae.py:6             VAE (decoder only)    */

typedef struct dmx_ctx dmx_ctx;
typedef struct dmx_model dmx_model;

int dmx_abi_version(void);
const char* dmx_last_error(void);

/* Context: one per device per process. */
int dmx_create(int device, dmx_ctx** out);
int dmx_destroy(dmx_ctx* ctx);

/* Sinusoidal time table pos[t-1][0..255] for t = 1..tmax (host fp32, computed by the
 * caller with the reference's own formula, models/unet_cond.py:155-161), copied to
 * the device. */
int dmx_set_time_table(dmx_ctx* ctx, const float* host_table, int tmax);

/* ---- weights (replaces Utils.loadModel -> load_state_dict, utils.py:68-73) ---------
 * Keys are the reference state_dict names; listing them needs no GPU. */
int dmx_model_num_keys(int kind, int in_ch, int remove_deep_conv);
int dmx_model_key(int kind, int in_ch, int remove_deep_conv, int index, char* name_out, int name_cap,
                  int64_t* shape_out /* [4] */, int* ndim_out);

int dmx_model_create(dmx_ctx* ctx, int kind, int in_ch, int remove_deep_conv, dmx_model** out);

/* Constructor arguments of the reference networks that change the checkpoint layout or
 * the arithmetic (UnetCond / UnetCondWithGeomHead / VAE __init__, reference
 * models/unet_cond.py:113, models/unet_cond_geom.py:31-49, models/vae.py:11).
 * dmx_model_create(..) is dmx_model_create_cfg with the reference defaults
 * (num_classes 3, geom_dim 12, geom_hidden 256, scale_factor 0.18215). */
typedef struct dmx_model_config {
  int kind;             /* DMX_UNET_COND_GEOM .. DMX_VAE */
  int in_ch;            /* U-Net latent channels, 1..4 */
  int remove_deep_conv; /* models/unet_cond.py:139-145 */
  int num_classes;      /* class_emb has num_classes + 1 rows (models/unet_cond.py:121) */
  int geom_dim;         /* GeomHead output width (models/unet_cond_geom.py:38) */
  int geom_hidden;      /* GeomHead hidden width (models/unet_cond_geom.py:39) */
  float scale_factor;   /* VAE latent scale (models/vae.py:11,59,66) */
} dmx_model_config;
int dmx_model_create_cfg(dmx_ctx* ctx, const dmx_model_config* cfg, dmx_model** out);
int dmx_model_cfg_num_keys(const dmx_model_config* cfg);
int dmx_model_cfg_key(const dmx_model_config* cfg, int index, char* name_out, int name_cap,
                      int64_t* shape_out /* [4] */, int* ndim_out);
int dmx_model_destroy(dmx_model* m);
/* Register one reference-layout tensor (device pointer, fp32 contiguous).  The pointer is
 * read by dmx_model_finalize and again by dmx_model_refresh and the training entry points, so
 * a caller using those keeps the tensor alive (and at the same address) for the model's life. */
int dmx_model_set_tensor(dmx_model* m, const char* name, const float* dev_ptr, const int64_t* shape, int ndim);
/* Repack every registered tensor into the model's kernel layouts (device-side). */
int dmx_model_finalize(dmx_model* m, void* stream);
/* The registered tensors changed in place (optimizer.step, load_state_dict's copy_): repeat
 * every repack on `stream` (no host sync); the split-precision planes are re-derived before the
 * next mode-1/2 launch.  Replaces re-running Utils.loadModel after each update (utils.py:68-73). */
int dmx_model_refresh(dmx_model* m, void* stream);
/* GEMM arithmetic: 0 = fp32 MFMA (exact fp32 products), 1 (default) = fp32 operands split
 * into fp16 hi+lo on the fp16 matrix cores (3 MFMAs, fp32 accumulate, ~1e-7 relative),
 * 2 = fp16 operands (BASELINE config 4: one MFMA, fp32 accumulate, fp32 norms/softmax/scheduler). */
int dmx_model_set_precision(dmx_model* m, int prec);
int dmx_model_get_precision(const dmx_model* m);
/* Range guard of the split-precision modes (1, 2): an operand beyond the f16 range turns a
 * network output (eps / decoded pixel / encoder head) non-finite, and the output kernels then
 * raise a sticky per-model flag.  Reads it (synchronising `stream`), optionally clearing it;
 * the Python samplers check it at chunk boundaries and recompute the chunk in mode 0. */
int dmx_model_range_check(dmx_model* m, int reset, int* flagged, void* stream);

/* ---- U-Net forward (replaces model(x, t, y, cond_vals, cond_mask), diff.py:149-150) --
 * x: (n,in_ch,h,w); t: (n,) int64 in [1, tmax]; y: (n,) int64 or NULL (DMX_UNET);
 * vals/mask: (n,12) or NULL; eps: (n,in_ch,h,w); geom: (n,12) or NULL. */
int dmx_unet_forward(dmx_model* m, const float* x, const int64_t* t, const int64_t* y, const float* vals,
                     const float* mask, float* eps, float* geom, int n, int h, int w, void* stream);

/* ---- one denoising step (replaces Diffuser.denoise_cond, diff.py:127-162, with the two
 * model calls batched as one 2n-sample forward, and Diffuser.denoise, diff.py:32-56) ----- */
typedef struct dmx_step_args {
  const float* x_in;        /* (n,C,h,w) */
  float* x_out;             /* (n,C,h,w); may alias x_in */
  const int64_t* t;         /* device; t_stride 0 => one value for every sample */
  int t_stride;
  const int64_t* y;         /* (n,) class ids, NULL for DMX_UNET */
  int64_t null_label;       /* diff.py:148 */
  const float* vals;        /* (n,12) or NULL */
  const float* mask;        /* (n,12) or NULL */
  float guidance;           /* > 0 => CFG (diff.py:147); DMX_UNET ignores it */
  const float* c1;          /* device tables [T]: (1-a)/sqrt(1-ab), sqrt(a), posterior std */
  const float* c2;
  const float* sd;
  int T;
  const float* noise;       /* (n,C,h,w) device noise, or NULL => on-device Philox */
  uint64_t seed;            /* Philox key (noise == NULL) */
  int64_t sample_offset;    /* global index of sample 0 (shard-invariant noise) */
  int n, h, w;
} dmx_step_args;

int dmx_step(dmx_model* m, const dmx_step_args* a, void* stream);

/* Run `steps` consecutive steps in place (x_in == x_out required), t taken from the
 * device scalar a->t (t_stride 0) and decremented on the device after each step; the
 * step is captured once into a hipGraph when use_graph != 0.  Noise must be NULL
 * (Philox).  This is the diff.py:332-344 loop without host round trips. */
int dmx_sample_loop(dmx_model* m, const dmx_step_args* a, int steps, int use_graph, void* stream);

/* Standalone K1 update (diff.py:151,158-162) for duck-typed foreign models:
 * eps = eu + g*(ec-eu) (ec NULL => eps = eu); x' = (x - c1*eps)/c2 + noise*sd. */
int dmx_ddpm_update(const float* x, float* x_out, const float* eu, const float* ec, float guidance,
                    const int64_t* t, int t_stride, const float* c1, const float* c2, const float* sd, int T,
                    const float* noise, uint64_t seed, int64_t sample_offset, int n, int c, int h, int w,
                    void* stream);

/* ---- VAE decode (replaces VAE.decode, vae.py:64-69, plus Diffuser.reverse_to_img's
 * x*255 -> clamp -> uint8, diff.py:58-62) ---------------------------------------------
 * z: (n,4,h,w); img: (n,3,8h,8w) fp32 or NULL; u8: (n,8h,8w,3) uint8 (HWC) or NULL. */
int dmx_vae_decode(dmx_model* m, const float* z, float* img, uint8_t* u8, int n, int h, int w, void* stream);

/* ---- latent-channel frames (replaces generate_steps.py:47-64 save_latent_channels_by_dir's
 * per-channel min-max -> *255 -> uint8 before the PNG write) ---------------------------------
 * z: (n,c,h,w) fp32 device; out: (n,c,h,w) uint8 device, byte-identical to the reference's. */
int dmx_latent_frames_u8(const float* z, uint8_t* out, int n, int c, int h, int w, void* stream);

/* ---- generated-image metrics (replaces eval_iou_noise.py:77-94 binarisation and 162-272
 * distance transform / compute_metrics) ------------------------------
 * gt, pred: (n,h,w) uint8 device — masks (0 / nonzero; gray = 0) or grayscale images binarised
 * here (gray = 1: foreground = v < threshold if invert else v >= threshold); h, w <= 16384.
 * workspace: n*h*w int32 device scratch; out: (n,9) float64 device =
 * {iou, gt_iou, far_noise_ratio, gauss_recall, inter, union, gt_area, pred_area, fp}. */
int dmx_eval_metrics(const uint8_t* gt, const uint8_t* pred, int n, int h, int w, int gray, int threshold, int invert,
                     double sigma, int* workspace, double* out, void* stream);

/* ---- VAE encode (replaces VAE.encode, vae.py:51-62) -------------
 * x: (n,3,h,w) fp32, h and w multiples of 8; eps: (n,4,h/8,w/8) = the reference's
 * torch.randn_like(std) draw (caller-drawn, so the global RNG stream matches);
 * z: (n,4,h/8,w/8) = (mu + eps * exp(0.5 logvar)) * 0.18215; kl: (n,) per-sample KL term
 * (VAE.encode's returned kl is kl.mean()). */
int dmx_vae_encode(dmx_model* m, const float* x, const float* eps, float* z, float* kl, int n, int h, int w,
                   void* stream);

/* ---- training step (replaces the forward + loss.backward() of UnetCondWithGeomHead / UnetCond
 * in train_latent_cond.py:148-162) ------------------------------------
 * dmx_train_forward: model(x, t, y, cond_vals, cond_mask) with fp32 semantics (x3 split GEMMs with
 * device-side scales whatever the model's precision), recording the activations the backward needs in a tape owned by the
 * model; x: (n,in_ch,h,w); t, y: (n,) int64 (t in [1, tmax], y in [0, num_classes]);
 * vals/mask: (n,12) or NULL; eps: (n,in_ch,h,w) out; geom: (n,geom_dim) out or NULL.
 * *tape_id identifies the tape (one per model: a later forward replaces it).
 * dmx_train_backward: d_eps (n,in_ch,h,w) = dLoss/deps, d_geom (n,geom_dim) = dLoss/dgeom
 * (either may be NULL = zero); writes dLoss/dparam for every state_dict key into grads[i]
 * (one device pointer per key in dmx_model_cfg_key order, each of that key's shape; keys whose
 * branch did not run — cond_mlp without vals — receive zeros).  No gradient for x. */
int dmx_train_forward(dmx_model* m, const float* x, const int64_t* t, const int64_t* y, const float* vals,
                      const float* mask, int n, int h, int w, float* eps, float* geom, int64_t* tape_id,
                      void* stream);
int dmx_train_backward(dmx_model* m, int64_t tape_id, const float* d_eps, const float* d_geom, float* const* grads,
                       int n_grads, void* stream);

/* ---- measurement: one eager step with a HIP event pair around every launch -----------
 * Fills up to `cap` records (kernel name as rocprofv3 shows it, layer label, algorithmic
 * FLOPs and HBM bytes of that launch, and its event-timed duration in ms). */
typedef struct dmx_kernel_record {
  char kernel[96];
  char layer[48];
  double flops;
  double bytes;
  float ms;
} dmx_kernel_record;

int dmx_step_profile(dmx_model* m, const dmx_step_args* a, dmx_kernel_record* recs, int cap, int* n_out,
                     void* stream);

/* ---- debugging: with taps enabled, dmx_unet_forward records every block output
 * (NHWC, inside the workspace) so they can be copied out and compared layer by layer. */
int dmx_debug_enable(dmx_model* m, int on);
int dmx_debug_num_taps(const dmx_model* m);
int dmx_debug_tap(dmx_model* m, int i, char* name_out, int cap, int64_t* count_out, float* dst, void* stream);

/* ---- multi-head attention core backward (the adjoint of nn.MultiheadAttention's softmax(Q K^T /
 * sqrt(D)) V core, models/unet_cond.py:36,49, 4 heads; used by dmx_train_backward, exported for its
 * test): qkv (n,L,3C) = q | k | v (head h at columns h*C/4), o = the core's output (n,L,C), dout =
 * dLoss/do (n,L,C); writes dLoss/dqkv (n,L,3C).  C/4 in {16, 32, 64}; all device fp32. */
int dmx_attn_core_backward(const float* qkv, const float* o, const float* dout, float* dqkv, int n, int L, int C,
                           void* stream);

/* ---- timing diagnostic (libraries built with -DDMX_DIAG=1 only; regular builds return 0): the
 * per-block s_memtime stamps of the Winograd conv launches ({start, after prologue, after chunk loop,
 * end, hardware id} x 2048 blocks x 32 launch slots, uint64) copied to host memory; returns the count
 * copied or -1; host == NULL resets the table and the launch counter.  tools/wino_stamps.py reads them. */
int dmx_diag_wino_stamps(unsigned long long* host, int cap);

/* Bytes of device workspace currently held by a model (diagnostics). */
int64_t dmx_model_workspace_bytes(const dmx_model* m);

#ifdef __cplusplus
}
#endif
#endif /* DMX_H_ */
