// dmx — training step of the conditional U-Net: the forward with a tape
// and the backward pass of UnetCond / UnetCondWithGeomHead, as train_latent_cond.py:136-163
// runs them (model(z_noisy, t, y, cond_vals, cond_mask) -> F.mse_loss + masked_geom_mse ->
// loss.backward(); the loss itself and Adam stay in torch).
//
// Forward = the inference trunk's kernels in exact-fp32 mode (fp32 MFMA implicit GEMMs, no
// deferred split-K fusion so every raw conv output is materialised) plus the few values the
// backward needs that inference never stores (pre-GELU FF activations, embedding MLP inputs).
// The tape lives in its own workspace (m->tws) until the matching dmx_train_backward.
// Backward (train.h kernels + the same fp32 implicit GEMM for data gradients):
//   GroupNorm / LayerNorm / GELU / SiLU / max-pool / bilinear-upsample adjoints, conv and Linear
//   data gradients as implicit GEMMs over flipped / transposed weights (packed once, refreshed
//   with the weights), weight gradients on fp32 MFMA (wgrad_kernel), attention core backward by
//   recomputation.  Parameter gradients are written in the reference's state_dict layout.
//
// Included by engine.hip after the inference engine (same translation unit).
#pragma once

namespace dmx {

struct TRes {  // one ResBlock of the training forward (models/unet_cond.py:10-30)
  const ResW* w = nullptr;
  int N = 0, H = 0, W = 0;
  bool residual = false;
  const float* x = nullptr;  // NHWC input (also the residual)
  float *r1 = nullptr, *a1 = nullptr, *r2 = nullptr, *out = nullptr;
  float2 *rp1 = nullptr, *rp2 = nullptr;
  int rr1 = 0, rr2 = 0;
  int emb_off = -1;  // >= 0: out += emb head slice (Down / Up, unet_cond.py:69,99)
};
struct TAttn {  // one AttenionBlock (models/unet_cond.py:32-52)
  const AttnW* w = nullptr;
  int N = 0, H = 0, W = 0;
  const float* x = nullptr;
  float *xl = nullptr, *qkv = nullptr, *ao = nullptr, *av = nullptr, *al = nullptr, *h1 = nullptr, *f = nullptr,
        *out = nullptr;
  float* st = nullptr;  // [N][4][L][3]: the forward's row max, 1 / sum (attention_kernel), the backward's Dlt
};
struct TUp {  // Up's bilinear x2 + pad + concat input (models/unet_cond.py:87-97)
  float* cat = nullptr;
  const float* skip = nullptr;
  const float* low = nullptr;
  int C0 = 0, C1 = 0, H = 0, W = 0, Hs = 0, Ws = 0, padT = 0, padL = 0;
};

struct Tape {
  int64_t id = 0;
  int n = 0, h = 0, w = 0;
  bool cond = false;  // cond_vals / cond_mask given (unet_cond_geom.py:91)
  int64_t* y = nullptr;
  float *xin = nullptr, *in24 = nullptr, *v0 = nullptr, *ca = nullptr, *ch = nullptr, *v = nullptr, *s = nullptr,
        *heads = nullptr;
  TRes inc;
  const float* skip[3] = {nullptr, nullptr, nullptr};
  int sh[3] = {0, 0, 0}, sw[3] = {0, 0, 0}, sc[3] = {0, 0, 0};
  float* pooled[3] = {nullptr, nullptr, nullptr};
  TRes dr0[3], dr1[3], bot[3], ur0[3], ur1[3];
  TAttn dsa[3], usa[3];
  TUp up[3];
  const float* feat = nullptr;
  float *g = nullptr, *hpre = nullptr, *hs = nullptr;
};

static int ew_blocks(size_t n) { return (int)std::min<size_t>((n + 255) / 256, 8192); }

static const float* srcp(dmx_model* m, const std::string& name) {
  auto it = m->inputs.find(name);
  if (it == m->inputs.end()) throw Error(DMX_E_STATE, "registered tensor '" + name + "' missing");
  return it->second.first;
}

// Gradient destinations, one per state_dict key (dmx_model_cfg_key order).
struct GradMap {
  std::map<std::string, float*> g;
  float* operator()(const std::string& name) const {
    auto it = g.find(name);
    if (it == g.end() || it->second == nullptr) throw Error(DMX_E_ARG, "no gradient buffer for '" + name + "'");
    return it->second;
  }
};

// Workspace run twice (plan: sizes only, then real) in a dedicated arena.
template <typename F>
static void run_arena(dmx_model* m, hipStream_t st, Arena& A, void*& mem, size_t& cap, F&& body) {
  A.base = nullptr;
  A.off = 0;
  A.plan = true;
  std::vector<size_t> trace;
  A.trace = check_args() ? &trace : nullptr;
  A.n = 0;
  {
    Run R{m, st, true, A};
    A.layer = &R.layer;
    body(R);
  }
  if (A.off > cap) {
    if (mem) {
      HIPCHK(hipStreamSynchronize(st));
      HIPCHK(hipFree(mem));
    }
    mem = nullptr;
    cap = 0;
    HIPCHK(hipMalloc(&mem, A.off));
    cap = A.off;
  }
  const size_t planned = A.off;
  poison(mem, A.off, st);
  A.base = static_cast<char*>(mem);
  A.off = 0;
  A.plan = false;
  A.n = 0;
  Run R{m, st, false, A};
  A.layer = &R.layer;
  try {
    body(R);
  } catch (...) {
    A.trace = nullptr;
    A.layer = nullptr;
    throw;
  }
  A.trace = nullptr;
  A.layer = nullptr;
  if (A.off != planned) throw Error(DMX_E_INTERNAL, "workspace plan / run mismatch");
}

// ---------------------------------------------------------------------------
// data-gradient weights (packed once on the first training call, refreshed with the rest)
// ---------------------------------------------------------------------------
// conv3x3 pad 1 [cout][cin] -> its data gradient: conv3x3 pad 1 over dY with the kernel flipped
// and the channel roles swapped (cin' = cout, cout' = cin); packed straight from the forward weight
// (RepackJob kind 3)
static ConvW pack_dgrad_conv(Packer& P, const std::string& wname, int cin, int cout) {
  ConvW c;
  c.cin = cout;
  c.cout = cin;
  c.taps = 9;
  c.kpad = rup(9 * cout, 64);
  c.npad = rup(cin, 128);
  c.B = P.alloc((size_t)c.npad * c.kpad);
  P.repack(c.B, P.in(wname).first, 3, 1, c.npad, c.kpad, cin, cout, 3);
  P.split_dev(c);
  return c;
}

// Linear [fout][fin] -> dX = dY W: a Linear with weight W^T [fin][fout] (RepackJob kind 4)
static ConvW pack_dgrad_linear(Packer& P, const std::string& wname, int fin, int fout) {
  ConvW c;
  c.cin = fout;
  c.cout = fin;
  c.taps = 1;
  c.kpad = rup(fout, 64);
  c.npad = rup(fin, 128);
  c.B = P.alloc((size_t)c.npad * c.kpad);
  P.repack(c.B, P.in(wname).first, 4, 1, c.npad, c.kpad, fin, fout, 1);
  P.split_dev(c);
  return c;
}

// the recorded device splits (Packer::split_dev) as two batched launches (the split over chunks of
// SPLIT_CHUNK elements, so every block carries the same work whatever the weight sizes)
static void run_split_jobs(dmx_model* m, hipStream_t st) {
  const size_t nj = m->split_jobs.size();
  if (nj == 0) return;
  if (m->split_table_n != nj) {
    std::vector<uint2> ch;
    for (size_t i = 0; i < nj; ++i) {
      if (m->split_jobs[i].n >= (1ull << 32)) throw Error(DMX_E_INTERNAL, "split: weight too large");
      for (size_t f = 0; f < m->split_jobs[i].n; f += SPLIT_CHUNK) ch.push_back(make_uint2((unsigned)i, (unsigned)f));
    }
    if (m->split_table) HIPCHK(hipFree(m->split_table));
    m->split_table = nullptr;
    HIPCHK(hipMalloc(&m->split_table, nj * sizeof(SplitJob) + ch.size() * sizeof(uint2)));
    HIPCHK(hipMemcpy(m->split_table, m->split_jobs.data(), nj * sizeof(SplitJob), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(static_cast<char*>(m->split_table) + nj * sizeof(SplitJob), ch.data(), ch.size() * sizeof(uint2),
                     hipMemcpyHostToDevice));
    m->split_table_n = nj;
    m->split_chunks = ch.size();
  }
  const SplitJob* t = static_cast<const SplitJob*>(m->split_table);
  const uint2* ch = reinterpret_cast<const uint2*>(t + nj);
  absmax_batch_kernel<<<dim3(SPLIT_PARTS, (unsigned)nj), 256, 0, st>>>(t);
  HIPCHK(hipGetLastError());
  split_batch_kernel<<<(unsigned)m->split_chunks, 256, 0, st>>>(t, ch);
  HIPCHK(hipGetLastError());
}

// The training forward's copy of a forward weight: the same packed fp32 B (refreshed with the model),
// its own f16 hi / lo planes split on the device with a device-side scale after every refresh (the
// inference planes keep their host-derived scale and are re-derived lazily), so the forward GEMMs run
// on the x3 split implicit GEMM; a weight the x3 kernel cannot take (Cin < 64: the padded input
// conv) keeps no planes and runs the exact-fp32 GEMM.
static ConvW fwd_x3_weight(Packer& P, const ConvW& c) {
  ConvW t = c;
  t.Bh = t.Bl = t.Fh = t.Fl = t.Uh = t.Ul = nullptr;
  t.inv_dev = nullptr;
  t.amax_dev = nullptr;
  if (c.cin >= 64 && c.phases == 1) P.split_dev(t);
  return t;
}

static void ensure_train(dmx_model* m, hipStream_t st) {
  if (m->train_ready) return;
  Packer P{m, st};
  auto res = [&](ResW& r, bool need_dx) {
    if (need_dx) r.d1 = pack_dgrad_conv(P, r.prefix + ".double_conv.0.weight", r.cin, r.mid);
    r.d2 = pack_dgrad_conv(P, r.prefix + ".double_conv.3.weight", r.mid, r.cout);
    r.t1 = fwd_x3_weight(P, r.c1);
    r.t2 = fwd_x3_weight(P, r.c2);
  };
  res(m->inc, false);  // the network input takes no gradient
  for (int i = 0; i < 3; ++i) {
    res(m->down[i].r0, true);
    res(m->down[i].r1, true);
    res(m->up[i].r0, true);
    res(m->up[i].r1, true);
  }
  for (int i = 0; i < m->nbot; ++i) res(m->bot[i], true);
  for (auto& a : m->sa) {
    const int c = a.c;
    a.dqkv = pack_dgrad_linear(P, a.prefix + ".mha.in_proj_weight", c, 3 * c);
    a.dout = pack_dgrad_linear(P, a.prefix + ".mha.out_proj.weight", c, c);
    a.df1 = pack_dgrad_linear(P, a.prefix + ".ff_self.1.weight", c, c);
    a.df2 = pack_dgrad_linear(P, a.prefix + ".ff_self.3.weight", c, c);
    a.tqkv = fwd_x3_weight(P, a.qkv);
    a.to = fwd_x3_weight(P, a.o);
    a.tf1 = fwd_x3_weight(P, a.f1);
    a.tf2 = fwd_x3_weight(P, a.f2);
  }
  run_split_jobs(m, st);
  HIPCHK(hipStreamSynchronize(st));
  m->train_ready = true;
}

// ---------------------------------------------------------------------------
// training forward
// ---------------------------------------------------------------------------
// C[I][J] (+)= A B (+ bias) through small_gemm_kernel (train.h), l split over grid.z until >= 256 blocks
static void small_gemm(Run& R, SmallGemm g) {
  const int tiles = cdiv(g.I, 32) * cdiv(g.J, 32);
  int splits = std::max(1, std::min(cdiv(256, tiles), cdiv(g.L, 64)));
  g.lsplit = cdiv(g.L, splits);
  splits = cdiv(g.L, g.lsplit);
  float* part = splits > 1 ? R.ws.get<float>((size_t)splits * g.I * g.J) : nullptr;
  if (R.plan) return;
  float* out = g.c;
  if (splits > 1) g.c = part;
  small_gemm_kernel<<<dim3(cdiv(g.J, 32), cdiv(g.I, 32), splits), 256, 0, R.st>>>(g);
  HIPCHK(hipGetLastError());
  if (splits > 1) {
    small_gemm_finish_kernel<<<ew_blocks((size_t)g.I * g.J), 256, 0, R.st>>>(part, splits, g.I, g.J, g.bias, out, g.ldc,
                                                                            g.accumulate);
    HIPCHK(hipGetLastError());
  }
}
// y[r][o] = b[o] + sum_k x[r][k] W[o][k]
static void dense_fwd(Run& R, const float* x, int ldx, const float* w, const float* b, int rows, int O, int K, float* y,
                      int ldy) {
  small_gemm(R, SmallGemm{x, w, ldx, 1, 1, K, rows, O, K, 0, y, ldy, b, 0});
}

static TRes train_res(Run& R, const ResW& w, const float* x, int N, int H, int W, bool residual, const float* emb,
                      int emb_stride, int emb_off) {
  TRes t;
  t.w = &w;
  t.N = N;
  t.H = H;
  t.W = W;
  t.residual = residual;
  t.x = x;
  const int M = N * H * W, HW = H * W, seg = 32;
  t.r1 = R.ws.get<float>((size_t)M * w.mid);
  t.rp1 = R.ws.get<float2>((size_t)M * (w.mid / seg));
  t.a1 = R.ws.get<float>((size_t)M * w.mid);
  t.r2 = R.ws.get<float>((size_t)M * w.cout);
  t.rp2 = R.ws.get<float2>((size_t)M * (w.cout / seg));
  t.out = R.ws.get<float>((size_t)M * w.cout);
  t.rr1 = gemm(R, plain_src(x, w.cin), SRC_PLAIN, N, H, W, w.t1, EPI_STATS, t.r1, nullptr, t.rp1, seg);
  NormParams n1 = norm_params(t.r1, t.rp1, w.mid / seg, t.rr1, w.g1.p, w.b1.p, w.mid, HW, t.a1);
  n1.act = 1;
  norm(R, n1, N);
  t.rr2 = gemm(R, plain_src(t.a1, w.mid), SRC_PLAIN, N, H, W, w.t2, EPI_STATS, t.r2, nullptr, t.rp2, seg);
  NormParams n2 = norm_params(t.r2, t.rp2, w.cout / seg, t.rr2, w.g2.p, w.b2.p, w.cout, HW, t.out);
  if (residual) n2.res = x;
  if (emb != nullptr) {
    n2.emb = emb;
    n2.emb_stride = emb_stride;
    n2.emb_off = emb_off;
    t.emb_off = emb_off;
  }
  norm(R, n2, N);
  return t;
}

static TAttn train_attn(Run& R, const AttnW& a, const float* x, int N, int H, int W) {
  TAttn t;
  t.w = &a;
  t.N = N;
  t.H = H;
  t.W = W;
  t.x = x;
  const int C = a.c, M = N * H * W, L = H * W;
  t.xl = R.ws.get<float>((size_t)M * C);
  t.qkv = R.ws.get<float>((size_t)M * 3 * C);
  t.ao = R.ws.get<float>((size_t)M * C);
  t.av = R.ws.get<float>((size_t)M * C);
  t.al = R.ws.get<float>((size_t)M * C);
  t.h1 = R.ws.get<float>((size_t)M * C);
  t.f = R.ws.get<float>((size_t)M * C);
  t.out = R.ws.get<float>((size_t)M * C);
  t.st = R.ws.get<float>((size_t)N * 4 * L * 3);
  layernorm(R, x, t.xl, a.l1w, a.l1b, M, C);
  gemm(R, plain_src(t.xl, C), SRC_PLAIN, N, H, W, a.tqkv, EPI_BIAS, t.qkv, nullptr, nullptr, 1);
  attention_core(R, t.qkv, t.ao, N, L, C, t.st);
  gemm(R, plain_src(t.ao, C), SRC_PLAIN, N, H, W, a.to, EPI_BIAS_RES, t.av, t.xl, nullptr, 1);
  layernorm(R, t.av, t.al, a.l2w, a.l2b, M, C);
  gemm(R, plain_src(t.al, C), SRC_PLAIN, N, H, W, a.tf1, EPI_BIAS, t.h1, nullptr, nullptr, 1);
  if (!R.plan) {
    gelu_fwd_kernel<<<ew_blocks((size_t)M * C), 256, 0, R.st>>>(t.h1, t.f, (size_t)M * C);
    HIPCHK(hipGetLastError());
  }
  gemm(R, plain_src(t.f, C), SRC_PLAIN, N, H, W, a.tf2, EPI_BIAS_RES, t.out, t.av, nullptr, 1);
  return t;
}

struct TrainArgs {
  const float* x;  // NCHW
  const int64_t* t;
  const int64_t* y;
  const float* vals;
  const float* mask;
  int n, h, w;
  float* eps;   // NCHW out
  float* geom;  // [n][geom_dim] out (UnetCondWithGeomHead) or null
};

static const char* kEmbHeads[6] = {"down1", "down2", "down3", "up1", "up2", "up3"};

static void emb_head_slices(dmx_model* m, int off[6], int hc[6]) {
  for (int i = 0; i < 3; ++i) {
    off[i] = m->down[i].emb_off;
    hc[i] = m->down[i].cout;
    off[3 + i] = m->up[i].emb_off;
    hc[3 + i] = m->up[i].cout;
  }
}

static void train_fwd_body(Run& R, Tape& T, const TrainArgs& a) {
  dmx_model* m = R.m;
  R.fwd_x3 = true;  // the ResW::t* / AttnW::t* weights (device-split planes) on the split GEMM
  const int N = a.n, H = a.h, W = a.w, HW = H * W;
  T.n = N;
  T.h = H;
  T.w = W;
  T.cond = a.vals != nullptr;
  T.xin = R.ws.get<float>((size_t)N * HW * m->inc.cin);
  T.y = R.ws.get<int64_t>(N);
  T.v0 = R.ws.get<float>((size_t)N * 256);
  T.v = R.ws.get<float>((size_t)N * 256);
  T.s = R.ws.get<float>((size_t)N * 256);
  T.heads = R.ws.get<float>((size_t)N * m->hsum);
  if (T.cond) {
    T.in24 = R.ws.get<float>((size_t)N * 24);
    T.ca = R.ws.get<float>((size_t)N * 256);
    T.ch = R.ws.get<float>((size_t)N * 256);
  }
  // embedding: emb = pos(t) + class_emb(y) (+ cond_mlp([vals, mask])), heads SiLU -> Linear
  // (models/unet_cond.py:155-167, unet_cond_geom.py:89-95, unet_cond.py:62-65 / 82-85)
  if (!R.plan) {
    R.layer = "train.embed";
    nchw_to_nhwc_kernel<<<ew_blocks((size_t)N * HW * m->inc.cin), 256, 0, R.st>>>(a.x, T.xin, N, m->in_ch,
                                                                                 m->inc.cin, HW);
    HIPCHK(hipMemcpyAsync(T.y, a.y, (size_t)N * sizeof(int64_t), hipMemcpyDeviceToDevice, R.st));
    embed_base_kernel<<<N, 256, 0, R.st>>>(a.t, T.y, m->ctx->pos_table, m->ctx->tmax, srcp(m, "class_emb.weight"),
                                           m->cfg.ncls, T.v0);
    HIPCHK(hipGetLastError());
  }
  if (T.cond) {
    if (!R.plan) {
      cat24_kernel<<<cdiv(N * 24, 256), 256, 0, R.st>>>(a.vals, a.mask, T.in24, N);
      HIPCHK(hipGetLastError());
    }
    dense_fwd(R, T.in24, 24, srcp(m, "cond_mlp.0.weight"), srcp(m, "cond_mlp.0.bias"), N, 256, 24, T.ca, 256);
    if (!R.plan) {
      silu_fwd_kernel<<<ew_blocks((size_t)N * 256), 256, 0, R.st>>>(T.ca, T.ch, (size_t)N * 256);
      HIPCHK(hipGetLastError());
    }
    dense_fwd(R, T.ch, 256, srcp(m, "cond_mlp.2.weight"), srcp(m, "cond_mlp.2.bias"), N, 256, 256, T.v, 256);
    if (!R.plan) {
      add_kernel<<<ew_blocks((size_t)N * 256), 256, 0, R.st>>>(T.v, T.v0, (size_t)N * 256);
      HIPCHK(hipGetLastError());
    }
  } else if (!R.plan) {
    HIPCHK(hipMemcpyAsync(T.v, T.v0, (size_t)N * 256 * sizeof(float), hipMemcpyDeviceToDevice, R.st));
  }
  if (!R.plan) {
    silu_fwd_kernel<<<ew_blocks((size_t)N * 256), 256, 0, R.st>>>(T.v, T.s, (size_t)N * 256);
    HIPCHK(hipGetLastError());
  }
  int off[6], hc[6];
  emb_head_slices(m, off, hc);
  for (int i = 0; i < 6; ++i) {
    const std::string p = std::string(kEmbHeads[i]) + ".emb_layer.1";
    dense_fwd(R, T.s, 256, srcp(m, p + ".weight"), srcp(m, p + ".bias"), N, hc[i], 256, T.heads + off[i], m->hsum);
  }
  // trunk (models/unet_cond_geom.py:52-76)
  R.layer = "train.inc";
  T.inc = train_res(R, m->inc, T.xin, N, H, W, false, nullptr, 0, 0);
  const float* cur = T.inc.out;
  int ch = H, cw = W, cc = 64;
  for (int i = 0; i < 3; ++i) {
    T.skip[i] = cur;
    T.sh[i] = ch;
    T.sw[i] = cw;
    T.sc[i] = cc;
    const int nh = ch / 2, nw = cw / 2;
    T.pooled[i] = R.ws.get<float>((size_t)N * nh * nw * cc);
    SrcDesc mp = plain_src(cur, cc);
    mp.Hs = ch;
    mp.Ws = cw;
    R.layer = "train.down" + std::to_string(i + 1);
    prep<SRC_MAXPOOL>(R, mp, T.pooled[i], N, nh, nw, "prep_kernel<2>");
    T.dr0[i] = train_res(R, m->down[i].r0, T.pooled[i], N, nh, nw, true, nullptr, 0, 0);
    T.dr1[i] = train_res(R, m->down[i].r1, T.dr0[i].out, N, nh, nw, false, T.heads, m->hsum, m->down[i].emb_off);
    cc = m->down[i].cout;
    ch = nh;
    cw = nw;
    R.layer = "train.sa" + std::to_string(i + 1);
    T.dsa[i] = train_attn(R, m->sa[i], T.dr1[i].out, N, ch, cw);
    cur = T.dsa[i].out;
  }
  for (int i = 0; i < m->nbot; ++i) {
    R.layer = "train.bot" + std::to_string(i + 1);
    T.bot[i] = train_res(R, m->bot[i], cur, N, ch, cw, false, nullptr, 0, 0);
    cur = T.bot[i].out;
    cc = m->bot[i].cout;
  }
  for (int i = 0; i < 3; ++i) {
    const int si = 2 - i;
    TUp& u = T.up[i];
    u.skip = T.skip[si];
    u.low = cur;
    u.C0 = T.sc[si];
    u.C1 = cc;
    u.H = T.sh[si];
    u.W = T.sw[si];
    u.Hs = ch;
    u.Ws = cw;
    const int dy = u.H - 2 * ch, dx = u.W - 2 * cw;
    u.padT = dy > 0 ? dy / 2 : 0;
    u.padL = dx > 0 ? dx / 2 : 0;
    SrcDesc us = plain_src(u.skip, u.C0 + u.C1);
    us.C0 = u.C0;
    us.src1 = cur;
    us.Hs = ch;
    us.Ws = cw;
    us.padT = u.padT;
    us.padL = u.padL;
    REQUIRE(us.C == m->up[i].r0.cin, "up: channel mismatch");
    u.cat = R.ws.get<float>((size_t)N * u.H * u.W * us.C);
    R.layer = "train.up" + std::to_string(i + 1);
    prep<SRC_UPCAT>(R, us, u.cat, N, u.H, u.W, "prep_kernel<3>");
    T.ur0[i] = train_res(R, m->up[i].r0, u.cat, N, u.H, u.W, true, nullptr, 0, 0);
    T.ur1[i] = train_res(R, m->up[i].r1, T.ur0[i].out, N, u.H, u.W, false, T.heads, m->hsum, m->up[i].emb_off);
    ch = u.H;
    cw = u.W;
    cc = m->up[i].cout;
    R.layer = "train.sa" + std::to_string(4 + i);
    T.usa[i] = train_attn(R, m->sa[3 + i], T.ur1[i].out, N, ch, cw);
    cur = T.usa[i].out;
  }
  T.feat = cur;
  // heads: out conv 1x1 (unet_cond.py:153) and GeomHead GAP -> Linear -> SiLU -> Linear
  const bool geom = m->kind == DMX_UNET_COND_GEOM;
  if (geom) {
    T.g = R.ws.get<float>((size_t)N * 64);
    T.hpre = R.ws.get<float>((size_t)N * m->cfg.ghid);
    T.hs = R.ws.get<float>((size_t)N * m->cfg.ghid);
  }
  R.layer = "train.heads";
  if (!R.plan) {
    out_head_kernel<<<dim3(cdiv(HW, 256), N), 256, 0, R.st>>>(T.feat, m->out_w, m->out_b, a.eps, m->in_ch, HW,
                                                              m->range_flag);
    HIPCHK(hipGetLastError());
  }
  if (geom) {  // (dense_fwd runs in the plan pass too: its split partials are workspace allocations)
    const int gh = m->cfg.ghid;
    if (!R.plan) {
      gap_fwd_kernel<<<N, 256, 0, R.st>>>(T.feat, HW, T.g);
      HIPCHK(hipGetLastError());
    }
    dense_fwd(R, T.g, 64, srcp(m, "geom_head.mlp.0.weight"), srcp(m, "geom_head.mlp.0.bias"), N, gh, 64, T.hpre, gh);
    if (!R.plan) {
      silu_fwd_kernel<<<ew_blocks((size_t)N * gh), 256, 0, R.st>>>(T.hpre, T.hs, (size_t)N * gh);
      HIPCHK(hipGetLastError());
    }
    if (a.geom != nullptr)
      dense_fwd(R, T.hs, gh, srcp(m, "geom_head.mlp.2.weight"), srcp(m, "geom_head.mlp.2.bias"), N, m->cfg.gdim, gh,
                a.geom, m->cfg.gdim);
  }
}

// ---------------------------------------------------------------------------
// backward building blocks
// ---------------------------------------------------------------------------
// out[c] = sum over `rows` rows of in[r * stride + c]: one pass for <= 256 rows, else row
// blocks of 256 into a partial table, then that table's column sums (fixed order).
// the final level of a column sum: deferred to colsum_flush (train_bwd_body's end) when R.colsum_defer
static void colsum_final(Run& R, const float* in, int rows, int C, size_t stride, float* outa, float* outb, int cb) {
  if (R.colsum_defer) {
    R.colsums.push_back(ColsumJob{in, outa, outb, stride, rows, C, cb});
    return;
  }
  colsum_kernel<<<dim3(cdiv(C, 64), 1), 256, 0, R.st>>>(in, rows, C, stride, rows, outa, 0, outb, cb);
  HIPCHK(hipGetLastError());
}

static void colsum_flush(Run& R) {
  for (size_t k = 0; k < R.colsums.size(); k += COLSUM_BATCH) {
    ColsumBatch b;
    std::memset(&b, 0, sizeof(b));
    const int nj = (int)std::min<size_t>(COLSUM_BATCH, R.colsums.size() - k);
    int cmax = 0;
    for (int i = 0; i < nj; ++i) {
      b.j[i] = R.colsums[k + i];
      cmax = std::max(cmax, b.j[i].C);
    }
    colsum_batch_kernel<<<dim3(cdiv(cmax, 64), nj), 256, 0, R.st>>>(b);
    HIPCHK(hipGetLastError());
  }
  R.colsums.clear();
}

static void colsum(Run& R, const float* in, int rows, int C, size_t stride, float* out) {
  const int rpb = 256, nb = cdiv(rows, rpb);
  float* part = nb > 1 ? R.ws.get<float>((size_t)nb * C) : nullptr;
  if (R.plan) return;
  if (nb == 1) {
    colsum_final(R, in, rows, C, stride, out, nullptr, 0);
  } else {
    colsum_kernel<<<dim3(cdiv(C, 64), nb), 256, 0, R.st>>>(in, rows, C, stride, rpb, part, 0);
    HIPCHK(hipGetLastError());
    colsum_final(R, part, nb, C, C, out, nullptr, 0);
  }
}

// outa[c] = sum of in[r][c], outb[c] = sum of in[r][C + c] (rows of 2C floats at `stride`): one launch
// per level instead of two colsum calls
static void colsum_pair(Run& R, const float* in, int rows, int C, size_t stride, float* outa, float* outb) {
  const int rpb = 256, nb = cdiv(rows, rpb);
  float* part = nb > 1 ? R.ws.get<float>((size_t)nb * 2 * C) : nullptr;
  if (R.plan) return;
  if (nb == 1) {
    colsum_final(R, in, rows, 2 * C, stride, outa, outb, C);
  } else {
    colsum_kernel<<<dim3(cdiv(2 * C, 64), nb), 256, 0, R.st>>>(in, rows, 2 * C, stride, rpb, part, 0);
    HIPCHK(hipGetLastError());
    colsum_final(R, part, nb, 2 * C, 2 * C, outa, outb, C);
  }
}

// bias gradient = column sums of dY [M][C]
static void bias_grad(Run& R, const float* dy, int M, int C, float* out) { colsum(R, dy, M, C, C, out); }

// Per-block partial maxima of |dY| for the device-side operand scale of the f16-core data and weight
// gradients (X3Params::a_amax, WgradParams::dy_amax).  The weight and data gradients of a layer read
// the same dY back to back (wgrad, then dgrad): the measurement is reused once, by the very next call
// on the same tensor, and then dropped — a later call on that buffer (its content may have changed)
// measures again.  Same decisions in the plan and the real pass (arena pointers correspond one to one).
static const unsigned* dy_amax(Run& R, const float* dy, size_t n, int* parts) {
  if (R.amax_src == dy && R.amax_n == n && R.amax_uses > 0) {
    if (--R.amax_uses == 0) R.amax_src = nullptr;
    *parts = R.amax_parts;
    return R.amax_slot;
  }
  const int np = (int)std::min<size_t>((n + 4095) / 4096, 256);  // (>= 4 float4 per thread)
  unsigned* slot = R.ws.get<unsigned>(256);
  if (!R.plan) {
    R.begin("absmax_part_kernel", 0.0, 4.0 * (double)n);
    absmax_part_kernel<<<np, 256, 0, R.st>>>(dy, n, slot);
    R.end();
    HIPCHK(hipGetLastError());
  }
  R.amax_src = dy;
  R.amax_n = n;
  R.amax_slot = slot;
  R.amax_parts = np;
  R.amax_uses = 1;
  *parts = np;
  return slot;
}

static bool wgrad_fast(int Cin, int Cout) { return Cin % 64 == 0 && Cout % 64 == 0; }

// weight gradient of a conv3x3 (taps 9) / Linear (taps 1) over NHWC input x and NHWC dY
static void wgrad(Run& R, const float* dy, const float* x, int N, int H, int W, int Cin, int Cout, int taps,
                  int cin_real, float* grad, float* bias_grad_out = nullptr) {
  const int M = N * H * W, K = taps * Cin;
  const bool fast = wgrad_fast(Cin, Cout);
  const int co_t = fast && Cout % 128 == 0 ? 128 : 64;  // wgrad_x3_kernel<128>: X staged once per 128 Cout
  const int bxy = cdiv(Cout, co_t) * cdiv(K, fast ? 128 : 64);
  // (the x3 kernel runs two 64 KB-LDS blocks per CU: one round of 512 blocks; fewer slabs for
  // wgrad_finish_kernel to read than the fp32 kernel's 1024-block target)
  // (the fp32 kernel's small-K / small-Cout layers — the padded input conv, the 1x1 out conv — have
  // one or two tiles: 64-row splits, so its launch is not a few hundred serial rows per block)
  int splits = std::max(1, std::min(cdiv(fast ? 512 : 1024, bxy), cdiv(M, fast ? 256 : 64)));
  const int rps = rup(cdiv(M, splits), 16);
  splits = cdiv(M, rps);
  float* part = R.ws.get<float>((size_t)splits * Cout * K);
  // bias gradient: column sums of dY, from the fast kernel's k-tile-0 blocks (per split)
  float* bpart = (bias_grad_out != nullptr && fast) ? R.ws.get<float>((size_t)splits * Cout) : nullptr;
  int nparts = 0;
  const unsigned* amax = fast ? dy_amax(R, dy, (size_t)M * Cout, &nparts) : nullptr;  // (x3 products)
  if (!R.plan) {
    check_range(R, dy, (size_t)M * Cout * 4, "wgrad dY");
    check_range(R, x, (size_t)M * Cin * 4, "wgrad X");
    WgradParams p{dy, x, N, H, W, Cin, Cout, taps, M, K, rps, part, bpart, amax, nparts};
    R.begin("wgrad_kernel", 2.0 * M * (double)Cout * K, 4.0 * ((double)M * (Cout + Cin) + (double)splits * Cout * K));
    if (fast && co_t == 128) wgrad_x3_kernel<128><<<dim3(Cout / 128, cdiv(K, 128), splits), 256, 0, R.st>>>(p);
    else if (fast) wgrad_x3_kernel<64><<<dim3(Cout / 64, cdiv(K, 128), splits), 256, 0, R.st>>>(p);
    else wgrad_kernel<<<dim3(cdiv(Cout, 64), cdiv(K, 64), splits), 256, 0, R.st>>>(p);
    R.end();
    HIPCHK(hipGetLastError());
    wgrad_finish_kernel<<<(int)(((size_t)Cout * K + 63) / 64), 256, 0, R.st>>>(part, splits, Cout, Cin, cin_real, taps, grad);
    HIPCHK(hipGetLastError());
  }
  // bias gradient = column sums of dY: the fast kernel's per-split sums, else a pass over dY
  if (bias_grad_out != nullptr) {
    if (fast) colsum(R, bpart, splits, Cout, Cout, bias_grad_out);
    else bias_grad(R, dy, M, Cout, bias_grad_out);
  }
}

// data gradient through a packed transposed / flipped weight: dx (+)= dY * W'
// On the f16 matrix cores (x3 split, fp32 accumulate): dY is scaled by a power of two from its own
// max|dY| before the split (gradients sit far below f16's normal range; unscaled, their lo parts went
// subnormal — 4.6e-4 rel-L2, round 2) and the weights carry a device-side scale refreshed with them
// (Packer::split_dev), so nothing waits on the host.
static void dgrad(Run& R, const float* dy, int Cy, int N, int H, int W, const ConvW& dw, float* dx, bool accumulate) {
  int parts = 0;
  const unsigned* amax = dy_amax(R, dy, (size_t)N * H * W * Cy, &parts);
  R.a_amax = amax;
  R.a_nparts = parts;
  try {
    gemm(R, plain_src(dy, Cy), SRC_PLAIN, N, H, W, dw, accumulate ? EPI_BIAS_RES : EPI_BIAS, dx,
         accumulate ? dx : nullptr, nullptr, 1);
  } catch (...) {
    R.a_amax = nullptr;
    R.a_nparts = 0;
    throw;
  }
  R.a_amax = nullptr;
  R.a_nparts = 0;
}

static void gn_bwd_launch(Run& R, const float* r, const float2* rp, int nseg, int rrows, const Vec& g, const Vec& b,
                          const float* res, int act, const float* dout, int N, int C, int HW, float* dr, float* dres,
                          int dres_mode, float* chpart, float* demb, int demb_stride, int demb_off,
                          int ppb, double* bsum, float* bch, unsigned* amax, int achunks);
static int gn_bwd_achunks(int HW, int C) { return std::max(1, std::min(64, cdiv(HW * C, 4096))); }

static void gn_bwd(Run& R, const float* r, const float2* rp, int nseg, int rrows, const Vec& g, const Vec& b,
                   const float* res, int act, const float* dout, int N, int C, int HW, float* dr, float* dres,
                   int dres_mode, float* ggamma, float* gbeta, float* demb, int demb_stride, int demb_off,
                   int amax_uses = 0) {
  // (the float4 passes: 4 channels per thread, C / 4 threads per pixel row dividing the 256-thread block)
  if (C % 4 != 0 || C / 4 > 256 || 256 % (C / 4) != 0) throw Error(DMX_E_INTERNAL, "gn_bwd: C must be 4 x a divisor of 256");
  // pass A over ~512 blocks in total (>= 16 pixels each)
  const int chunks = std::max(1, std::min(cdiv(512, N), cdiv(HW, 16)));
  const int ppb = cdiv(HW, chunks);
  float* chpart = R.ws.get<float>((size_t)N * 2 * C);
  double* bsum = R.ws.get<double>((size_t)N * chunks * 2);
  float* bch = R.ws.get<float>((size_t)N * chunks * 3 * C);
  // amax_uses > 0: pass B also writes the per-block max |dr| — the next amax_uses x3 gradient GEMMs
  // reading dr take their device-side scale from it (dy_amax) instead of a separate absmax pass
  const int achunks = gn_bwd_achunks(HW, C);
  unsigned* amax = amax_uses > 0 ? R.ws.get<unsigned>((size_t)N * achunks) : nullptr;
  if (!R.plan) gn_bwd_launch(R, r, rp, nseg, rrows, g, b, res, act, dout, N, C, HW, dr, dres, dres_mode, chpart,
                             demb, demb_stride, demb_off, ppb, bsum, bch, amax, achunks);
  if (amax_uses > 0) {
    R.amax_src = dr;
    R.amax_n = (size_t)N * HW * C;
    R.amax_slot = amax;
    R.amax_parts = N * achunks;
    R.amax_uses = amax_uses;
  }
  colsum_pair(R, chpart, N, C, 2 * (size_t)C, ggamma, gbeta);
}

static void gn_bwd_launch(Run& R, const float* r, const float2* rp, int nseg, int rrows, const Vec& g, const Vec& b,
                          const float* res, int act, const float* dout, int N, int C, int HW, float* dr, float* dres,
                          int dres_mode, float* chpart, float* demb, int demb_stride, int demb_off,
                          int ppb, double* bsum, float* bch, unsigned* amax, int achunks) {
  GnBwdParams p;
  std::memset(&p, 0, sizeof(p));
  p.r = r;
  p.rowpart = rp;
  p.nseg = nseg;
  p.rrows = rrows;
  p.gamma = g.p;
  p.beta = b.p;
  p.res = res;
  p.act = act;
  p.dout = dout;
  p.C = C;
  p.HW = HW;
  p.dr = dr;
  p.dres = dres;
  p.dres_mode = dres_mode;
  p.chpart = chpart;
  p.demb = demb;
  p.demb_stride = demb_stride;
  p.demb_off = demb_off;
  p.chunks = cdiv(HW, ppb);
  p.ppb = ppb;
  p.bsum = bsum;
  p.bch = bch;
  R.begin("gn_bwd_reduce_kernel", 0.0, 4.0 * (double)N * HW * C * (res ? 3 : 2));
  gn_bwd_reduce_kernel<<<dim3(p.chunks, N), 256, 0, R.st>>>(p);
  R.end();
  HIPCHK(hipGetLastError());
  p.amax_part = amax;
  R.begin("gn_bwd_apply_kernel", 0.0, 4.0 * (double)N * HW * C * (res ? 4 : 3));
  gn_bwd_apply_kernel<<<dim3(achunks, N), 256, 0, R.st>>>(p);
  R.end();
  HIPCHK(hipGetLastError());
}

static void ln_bwd(Run& R, const float* x, const Vec& w, const float* dy, float* dx, bool accumulate, int M, int C,
                   float* gw, float* gb) {
  const int blocks = std::min(cdiv(M, 4), 512);
  float* part = R.ws.get<float>((size_t)blocks * 2 * C);
  if (!R.plan) {
    R.begin("ln_bwd_kernel", 0.0, 4.0 * (double)M * C * 3);
    switch (C) {
      case 64: ln_bwd_kernel<1><<<blocks, 256, 0, R.st>>>(x, w.p, dy, dx, accumulate ? 1 : 0, part, M); break;
      case 128: ln_bwd_kernel<2><<<blocks, 256, 0, R.st>>>(x, w.p, dy, dx, accumulate ? 1 : 0, part, M); break;
      case 256: ln_bwd_kernel<4><<<blocks, 256, 0, R.st>>>(x, w.p, dy, dx, accumulate ? 1 : 0, part, M); break;
      default: throw Error(DMX_E_INTERNAL, "ln_bwd: unsupported C");
    }
    R.end();
    HIPCHK(hipGetLastError());
  }
  colsum_pair(R, part, blocks, C, 2 * (size_t)C, gw, gb);
}

// the two MFMA attention-backward launches (train.h); st: [N][4][L][3] — with have_stats, slots 0 / 1
// hold the forward's row max and 1 / sum (attention_kernel), else the dq kernel derives them first
static void attn_core_bwd_launch(const float* qkv, const float* o, const float* dout, float* dqkv, float* st, int N,
                                 int L, int C, bool have_stats, hipStream_t s) {
  const int D = C / 4;
  const dim3 grid(cdiv(L, 64), 4, N);
#define DMX_ATTB(DD)                                                                                   \
  if (have_stats) attn_dq_mfma_kernel<DD, false><<<grid, 256, 0, s>>>(qkv, o, dout, st, dqkv, L, C);  \
  else attn_dq_mfma_kernel<DD, true><<<grid, 256, 0, s>>>(qkv, o, dout, st, dqkv, L, C);              \
  attn_dkv_mfma_kernel<DD><<<grid, 256, 0, s>>>(qkv, dout, st, dqkv, L, C);
  switch (D) {
    case 16: DMX_ATTB(16) break;
    case 32: DMX_ATTB(32) break;
    case 64: DMX_ATTB(64) break;
    default: throw Error(DMX_E_INTERNAL, "attention backward: unsupported head dim");
  }
#undef DMX_ATTB
  HIPCHK(hipGetLastError());
}

// st: the training forward's statistics (TAttn::st)
static void attn_core_bwd(Run& R, const float* qkv, const float* o, const float* dout, float* dqkv, float* st, int N,
                          int L, int C) {
  if (R.plan) return;
  R.begin("attn_bwd_kernels<" + std::to_string(C / 4) + ">", 4.0 * 4.0 * N * (double)L * L * C,
          4.0 * N * (double)L * 6 * C);
  attn_core_bwd_launch(qkv, o, dout, dqkv, st, N, L, C, true, R.st);
  R.end();
}

// ResBlock backward: dout -> dx (x's gradient; accumulated when dx_acc), parameter gradients,
// and the emb slice's per-sample sums into demb (Down / Up second block).
static void res_bwd(Run& R, const TRes& t, const GradMap& G, const float* dout, float* dx, bool dx_acc, float* demb,
                    int demb_stride) {
  const ResW& w = *t.w;
  const int N = t.N, H = t.H, W = t.W, M = N * H * W, HW = H * W, seg = 32;
  const std::string& p = w.prefix;
  float* dr2 = R.ws.get<float>((size_t)M * w.cout);
  gn_bwd(R, t.r2, t.rp2, w.cout / seg, t.rr2, w.g2, w.b2, t.residual ? t.x : nullptr, 0, dout, N, w.cout, HW, dr2,
         t.residual ? dx : nullptr, t.residual ? (dx_acc ? 2 : 1) : 0, G(p + ".double_conv.4.weight"),
         G(p + ".double_conv.4.bias"), t.emb_off >= 0 ? demb : nullptr, demb_stride, t.emb_off,
         (wgrad_fast(w.mid, w.cout) ? 1 : 0) + 1);
  wgrad(R, dr2, t.a1, N, H, W, w.mid, w.cout, 9, w.mid, G(p + ".double_conv.3.weight"));
  float* da1 = R.ws.get<float>((size_t)M * w.mid);
  dgrad(R, dr2, w.cout, N, H, W, w.d2, da1, false);
  float* dr1 = R.ws.get<float>((size_t)M * w.mid);
  gn_bwd(R, t.r1, t.rp1, w.mid / seg, t.rr1, w.g1, w.b1, nullptr, 1, da1, N, w.mid, HW, dr1, nullptr, 0,
         G(p + ".double_conv.1.weight"), G(p + ".double_conv.1.bias"), nullptr, 0, 0,
         (wgrad_fast(w.cin, w.mid) ? 1 : 0) + (dx != nullptr ? 1 : 0));
  wgrad(R, dr1, t.x, N, H, W, w.cin, w.mid, 9, w.cin_real, G(p + ".double_conv.0.weight"));
  if (dx != nullptr) dgrad(R, dr1, w.mid, N, H, W, w.d1, dx, t.residual || dx_acc);
}

// AttenionBlock backward; dout (the block output's gradient) is consumed (used as scratch).
static void attn_bwd(Run& R, const TAttn& t, const GradMap& G, float* dout, float* dx) {
  const AttnW& a = *t.w;
  const int C = a.c, N = t.N, H = t.H, W = t.W, M = N * H * W, L = H * W;
  const std::string& p = a.prefix;
  // out = ff2(gelu(ff1(al))) + av
  wgrad(R, dout, t.f, N, H, W, C, C, 1, C, G(p + ".ff_self.3.weight"), G(p + ".ff_self.3.bias"));
  float* dh = R.ws.get<float>((size_t)M * C);
  dgrad(R, dout, C, N, H, W, a.df2, dh, false);
  if (!R.plan) {
    gelu_bwd_kernel<<<ew_blocks((size_t)M * C), 256, 0, R.st>>>(dh, t.h1, dh, (size_t)M * C);
    HIPCHK(hipGetLastError());
  }
  wgrad(R, dh, t.al, N, H, W, C, C, 1, C, G(p + ".ff_self.1.weight"), G(p + ".ff_self.1.bias"));
  float* dal = R.ws.get<float>((size_t)M * C);
  dgrad(R, dh, C, N, H, W, a.df1, dal, false);
  // al = LN2(av): dav = dout + LN2^T(dal)
  ln_bwd(R, t.av, a.l2w, dal, dout, true, M, C, G(p + ".ff_self.0.weight"), G(p + ".ff_self.0.bias"));
  float* dav = dout;
  // av = out_proj(attn(xl)) + xl
  wgrad(R, dav, t.ao, N, H, W, C, C, 1, C, G(p + ".mha.out_proj.weight"), G(p + ".mha.out_proj.bias"));
  float* dao = R.ws.get<float>((size_t)M * C);
  dgrad(R, dav, C, N, H, W, a.dout, dao, false);
  float* dqkv = R.ws.get<float>((size_t)M * 3 * C);
  attn_core_bwd(R, t.qkv, t.ao, dao, dqkv, t.st, N, L, C);
  wgrad(R, dqkv, t.xl, N, H, W, C, 3 * C, 1, C, G(p + ".mha.in_proj_weight"), G(p + ".mha.in_proj_bias"));
  dgrad(R, dqkv, 3 * C, N, H, W, a.dqkv, dav, true);  // dxl = dav + in_proj^T(dqkv)
  ln_bwd(R, t.x, a.l1w, dav, dx, false, M, C, G(p + ".ln.weight"), G(p + ".ln.bias"));
}

static void zero_grad(Run& R, const GradMap& G, dmx_model* m, const std::string& name) {
  if (R.plan) return;
  for (auto& k : m->keys)
    if (k.name == name) {
      size_t n = 1;
      for (auto s : k.shape) n *= (size_t)s;
      HIPCHK(hipMemsetAsync(G(name), 0, n * sizeof(float), R.st));
    }
}

// dW[o][k] = sum_r dY[r][o] x[r][k], db[o] = sum_r dY[r][o]
static void dense_dw(Run& R, const float* dy, int ldy, const float* x, int ldx, int rows, int O, int K, float* dw,
                     float* db) {
  small_gemm(R, SmallGemm{dy, x, 1, ldy, ldx, 1, O, K, rows, 0, dw, K, nullptr, 0});
  if (R.plan || db == nullptr) return;
  dense_db_kernel<<<cdiv(O, 256), 256, 0, R.st>>>(dy, ldy, rows, O, db);
  HIPCHK(hipGetLastError());
}
// dX[r][k] (+)= sum_o dY[r][o] W[o][k]
static void dense_dx(Run& R, const float* dy, int ldy, const float* w, int rows, int O, int K, float* dx, int ldx,
                     bool accumulate) {
  small_gemm(R, SmallGemm{dy, w, ldy, 1, K, 1, rows, K, O, 0, dx, ldx, nullptr, accumulate ? 1 : 0});
}

static void train_bwd_body(Run& R, Tape& T, const GradMap& G, const float* d_eps, const float* d_geom) {
  dmx_model* m = R.m;
  R.colsum_defer = !R.plan;  // the final-level column sums run batched at the end (colsum_flush)
  const int N = T.n, H = T.h, W = T.w, HW = H * W, M = N * HW, Co = m->in_ch;
  // heads
  R.layer = "train.heads.bwd";
  float* dfeat = R.ws.get<float>((size_t)M * 64);
  float* dyo = R.ws.get<float>((size_t)M * Co);
  if (!R.plan) {
    if (d_eps != nullptr) {
      nchw_to_nhwc_kernel<<<ew_blocks((size_t)M * Co), 256, 0, R.st>>>(d_eps, dyo, N, Co, Co, HW);
    } else {
      HIPCHK(hipMemsetAsync(dyo, 0, (size_t)M * Co * sizeof(float), R.st));
    }
    HIPCHK(hipGetLastError());
  }
  wgrad(R, dyo, T.feat, N, H, W, 64, Co, 1, 64, G("out.weight"), G("out.bias"));
  dense_dx(R, dyo, Co, srcp(m, "out.weight"), M, Co, 64, dfeat, 64, false);
  if (m->kind == DMX_UNET_COND_GEOM) {
    const int gh = m->cfg.ghid, gd = m->cfg.gdim;
    float* dhs = R.ws.get<float>((size_t)N * gh);
    float* dg = R.ws.get<float>((size_t)N * 64);
    if (d_geom != nullptr) {
      dense_dw(R, d_geom, gd, T.hs, gh, N, gd, gh, G("geom_head.mlp.2.weight"), G("geom_head.mlp.2.bias"));
      dense_dx(R, d_geom, gd, srcp(m, "geom_head.mlp.2.weight"), N, gd, gh, dhs, gh, false);
      if (!R.plan) {
        silu_bwd_kernel<<<ew_blocks((size_t)N * gh), 256, 0, R.st>>>(dhs, T.hpre, dhs, (size_t)N * gh, 0);
        HIPCHK(hipGetLastError());
      }
      dense_dw(R, dhs, gh, T.g, 64, N, gh, 64, G("geom_head.mlp.0.weight"), G("geom_head.mlp.0.bias"));
      dense_dx(R, dhs, gh, srcp(m, "geom_head.mlp.0.weight"), N, gh, 64, dg, 64, false);
      if (!R.plan) {
        gap_bwd_kernel<<<ew_blocks((size_t)M * 64), 256, 0, R.st>>>(dg, N, HW, dfeat);
        HIPCHK(hipGetLastError());
      }
    } else {
      for (const char* k : {"geom_head.mlp.0.weight", "geom_head.mlp.0.bias", "geom_head.mlp.2.weight",
                            "geom_head.mlp.2.bias"})
        zero_grad(R, G, m, k);
    }
  }
  float* demb = R.ws.get<float>((size_t)N * m->hsum);
  float* dskip[3];
  for (int i = 0; i < 3; ++i) dskip[i] = R.ws.get<float>((size_t)N * T.sh[i] * T.sw[i] * T.sc[i]);
  // up path, last block first
  float* dcur = dfeat;
  for (int i = 2; i >= 0; --i) {
    const int si = 2 - i;
    const TUp& u = T.up[i];
    const int Mi = N * u.H * u.W, Cin = u.C0 + u.C1;
    R.layer = "train.up" + std::to_string(i + 1) + ".bwd";
    float* dxs = R.ws.get<float>((size_t)Mi * m->up[i].cout);
    attn_bwd(R, T.usa[i], G, dcur, dxs);
    float* dh0 = R.ws.get<float>((size_t)Mi * Cin);
    res_bwd(R, T.ur1[i], G, dxs, dh0, false, demb, m->hsum);
    float* dcat = R.ws.get<float>((size_t)Mi * Cin);
    res_bwd(R, T.ur0[i], G, dh0, dcat, false, nullptr, 0);
    float* dlow = R.ws.get<float>((size_t)N * u.Hs * u.Ws * u.C1);
    if (!R.plan) {
      const size_t tot = (size_t)Mi * u.C0 + (size_t)N * u.Hs * u.Ws * u.C1;
      upcat_bwd_kernel<<<ew_blocks(tot), 256, 0, R.st>>>(dcat, dskip[si], dlow, N, u.H, u.W, u.C0, u.C1, u.Hs, u.Ws,
                                                         u.padT, u.padL, 0, 0);
      HIPCHK(hipGetLastError());
    }
    dcur = dlow;
  }
  for (int i = m->nbot - 1; i >= 0; --i) {
    R.layer = "train.bot" + std::to_string(i + 1) + ".bwd";
    const TRes& b = T.bot[i];
    float* d = R.ws.get<float>((size_t)b.N * b.H * b.W * b.w->cin);
    res_bwd(R, b, G, dcur, d, false, nullptr, 0);
    dcur = d;
  }
  for (int i = 2; i >= 0; --i) {
    R.layer = "train.down" + std::to_string(i + 1) + ".bwd";
    const TRes& r1 = T.dr1[i];
    const int Mi = N * r1.H * r1.W, Cin = T.sc[i];
    float* dxs = R.ws.get<float>((size_t)Mi * m->down[i].cout);
    attn_bwd(R, T.dsa[i], G, dcur, dxs);
    float* dh0 = R.ws.get<float>((size_t)Mi * Cin);
    res_bwd(R, r1, G, dxs, dh0, false, demb, m->hsum);
    float* dpool = R.ws.get<float>((size_t)Mi * Cin);
    res_bwd(R, T.dr0[i], G, dh0, dpool, false, nullptr, 0);
    if (!R.plan) {
      maxpool_bwd_kernel<<<ew_blocks((size_t)N * T.sh[i] * T.sw[i] * Cin), 256, 0, R.st>>>(
          T.skip[i], dpool, dskip[i], N, T.sh[i], T.sw[i], Cin, 1);
      HIPCHK(hipGetLastError());
    }
    dcur = dskip[i];
  }
  R.layer = "train.inc.bwd";
  res_bwd(R, T.inc, G, dcur, nullptr, false, nullptr, 0);
  // embedding
  R.layer = "train.embed.bwd";
  float* ds = R.ws.get<float>((size_t)N * 256);
  float* dv = R.ws.get<float>((size_t)N * 256);
  int off[6], hc[6];
  emb_head_slices(m, off, hc);
  for (int i = 0; i < 6; ++i) {
    const std::string p = std::string(kEmbHeads[i]) + ".emb_layer.1";
    dense_dw(R, demb + off[i], m->hsum, T.s, 256, N, hc[i], 256, G(p + ".weight"), G(p + ".bias"));
    dense_dx(R, demb + off[i], m->hsum, srcp(m, p + ".weight"), N, hc[i], 256, ds, 256, i > 0);
  }
  if (!R.plan) {
    silu_bwd_kernel<<<ew_blocks((size_t)N * 256), 256, 0, R.st>>>(ds, T.v, dv, (size_t)N * 256, 0);
    class_emb_bwd_kernel<<<m->cfg.ncls, 256, 0, R.st>>>(dv, T.y, N, m->cfg.ncls, G("class_emb.weight"));
    HIPCHK(hipGetLastError());
  }
  if (T.cond) {
    float* dch = R.ws.get<float>((size_t)N * 256);
    dense_dw(R, dv, 256, T.ch, 256, N, 256, 256, G("cond_mlp.2.weight"), G("cond_mlp.2.bias"));
    dense_dx(R, dv, 256, srcp(m, "cond_mlp.2.weight"), N, 256, 256, dch, 256, false);
    if (!R.plan) {
      silu_bwd_kernel<<<ew_blocks((size_t)N * 256), 256, 0, R.st>>>(dch, T.ca, dch, (size_t)N * 256, 0);
      HIPCHK(hipGetLastError());
    }
    dense_dw(R, dch, 256, T.in24, 24, N, 256, 24, G("cond_mlp.0.weight"), G("cond_mlp.0.bias"));
  } else {
    for (const char* k : {"cond_mlp.0.weight", "cond_mlp.0.bias", "cond_mlp.2.weight", "cond_mlp.2.bias"})
      zero_grad(R, G, m, k);
  }
  if (!R.plan) colsum_flush(R);
  R.colsum_defer = false;
}

static void check_train(dmx_model* m, int n, int h, int w) {
  check_shapes(m, n, h, w);
  REQUIRE(m->kind == DMX_UNET_COND_GEOM || m->kind == DMX_UNET_COND,
          "training is implemented for UnetCond / UnetCondWithGeomHead");
}

// Run body with the model in exact-fp32 GEMM mode (restored afterwards).
template <typename F>
static void with_fp32(dmx_model* m, F&& f) {
  const int prec = m->prec;
  m->prec = 0;
  try {
    f();
  } catch (...) {
    m->prec = prec;
    throw;
  }
  m->prec = prec;
}

// Replays the packing after in-place parameter updates: all parameter copies in one launch, the
// recorded jobs in order (padding / flip / transpose staging), then all repacks in one launch.
static void refresh_model(dmx_model* m, hipStream_t st) {
  if (!m->finalized) throw Error(DMX_E_STATE, "model weights not finalized");
  const size_t nc = m->copies.size(), nr = m->repacks.size();
  if (m->job_tables_n != nc + nr) {  // (re)upload the tables (training adds repacks after finalize)
    std::vector<BatchChunk> cc, rc;
    for (size_t i = 0; i < nc; ++i)
      for (size_t f = 0; f < m->copies[i].n; f += BATCH_CHUNK) cc.push_back(BatchChunk{(unsigned)i, (unsigned)f});
    std::vector<RepackTile> tc;
    for (size_t i = 0; i < nr; ++i) {
      const RepackJob& r = m->repacks[i];
      const size_t total = (size_t)r.P * r.Npad * r.Kpad;
      if (total >= (1ull << 32)) throw Error(DMX_E_INTERNAL, "refresh: weight too large for 32-bit repack");
      if ((r.kind == 0 || r.kind == 3) && r.KS == 3 && r.P == 1) {  // LDS-tiled (live region only)
        for (int n0 = 0; n0 < r.Cout; n0 += 16)
          for (int c0 = 0; c0 < r.Cin; c0 += 32) tc.push_back(RepackTile{(unsigned)i, (unsigned)n0, (unsigned)c0});
        continue;
      }
      for (size_t f = 0; f < total; f += BATCH_CHUNK) rc.push_back(BatchChunk{(unsigned)i, (unsigned)f});
    }
    if (m->job_tables) HIPCHK(hipFree(m->job_tables));
    m->job_tables = nullptr;
    const size_t b0 = nc * sizeof(CopyJob), b1 = nr * sizeof(RepackJob), b2 = cc.size() * sizeof(BatchChunk),
                 b3 = rc.size() * sizeof(BatchChunk), b4 = tc.size() * sizeof(RepackTile);
    HIPCHK(hipMalloc(&m->job_tables, b0 + b1 + b2 + b3 + b4 + 16));
    char* t = static_cast<char*>(m->job_tables);
    HIPCHK(hipMemcpy(t, m->copies.data(), b0, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t + b0, m->repacks.data(), b1, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t + b0 + b1, cc.data(), b2, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t + b0 + b1 + b2, rc.data(), b3, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(t + b0 + b1 + b2 + b3, tc.data(), b4, hipMemcpyHostToDevice));
    m->job_tables_n = nc + nr;
    m->copy_chunks = cc.size();
    m->repack_chunks = rc.size();
    m->repack_tiles = tc.size();
  }
  const char* t = static_cast<const char*>(m->job_tables);
  const CopyJob* ct = reinterpret_cast<const CopyJob*>(t);
  const RepackJob* rt = reinterpret_cast<const RepackJob*>(t + nc * sizeof(CopyJob));
  const BatchChunk* cch = reinterpret_cast<const BatchChunk*>(t + nc * sizeof(CopyJob) + nr * sizeof(RepackJob));
  const BatchChunk* rch = cch + m->copy_chunks;
  const RepackTile* rtl = reinterpret_cast<const RepackTile*>(rch + m->repack_chunks);
  if (m->copy_chunks) {
    copy_batch_kernel<<<(unsigned)m->copy_chunks, 256, 0, st>>>(ct, cch);
    HIPCHK(hipGetLastError());
  }
  for (auto& f : m->jobs) f(st);
  if (m->repack_chunks) {
    repack_batch_kernel<<<(unsigned)m->repack_chunks, 256, 0, st>>>(rt, rch);
    HIPCHK(hipGetLastError());
  }
  if (m->repack_tiles) {
    repack_tile_kernel<<<(unsigned)m->repack_tiles, 256, 0, st>>>(rt, rtl);
    HIPCHK(hipGetLastError());
  }
  run_split_jobs(m, st);  // device-side splits of the data-gradient weights
  m->planes_stale = true;
}

}  // namespace dmx
