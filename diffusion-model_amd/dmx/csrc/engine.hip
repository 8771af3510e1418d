// dmx engine: weights, workspace planning, U-Net / VAE orchestration, hipGraph
// step loop and the C ABI of include/dmx.h.
#include "dmx.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"
#include "igemm.h"
#include "igemm_x3.h"
#include "kernels.h"
#include "igemm_pp.h"
#include "launch.h"
#include "igemm_halo.h"
#include "tokmlp.h"
#include "eval.h"
#include "train.h"

namespace dmx {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
static thread_local std::string g_err;

#define HIPCHK(x)                                                                               \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) throw Error(DMX_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)
#define REQUIRE(c, msg)                                    \
  do {                                                     \
    if (!(c)) throw Error(DMX_E_ARG, std::string(msg));    \
  } while (0)

static inline int rup(int a, int b) { return (a + b - 1) / b * b; }
static inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// ===========================================================================
// Reference state_dict key lists (mirror of dmx/spec.py; the checkpoint contract
// of Utils.loadModel, utils.py:68-73).
// ===========================================================================
struct Key {
  std::string name;
  std::vector<int64_t> shape;
};
using Keys = std::vector<Key>;

static void k_res(Keys& k, const std::string& p, int cin, int cout, int mid = 0) {
  mid = mid ? mid : cout;
  k.push_back({p + ".double_conv.0.weight", {mid, cin, 3, 3}});
  k.push_back({p + ".double_conv.1.weight", {mid}});
  k.push_back({p + ".double_conv.1.bias", {mid}});
  k.push_back({p + ".double_conv.3.weight", {cout, mid, 3, 3}});
  k.push_back({p + ".double_conv.4.weight", {cout}});
  k.push_back({p + ".double_conv.4.bias", {cout}});
}
static void k_lin(Keys& k, const std::string& p, int fin, int fout) {
  k.push_back({p + ".weight", {fout, fin}});
  k.push_back({p + ".bias", {fout}});
}
static void k_attn(Keys& k, const std::string& p, int c) {
  k.push_back({p + ".mha.in_proj_weight", {3 * c, c}});
  k.push_back({p + ".mha.in_proj_bias", {3 * c}});
  k.push_back({p + ".mha.out_proj.weight", {c, c}});
  k.push_back({p + ".mha.out_proj.bias", {c}});
  k.push_back({p + ".ln.weight", {c}});
  k.push_back({p + ".ln.bias", {c}});
  k.push_back({p + ".ff_self.0.weight", {c}});
  k.push_back({p + ".ff_self.0.bias", {c}});
  k_lin(k, p + ".ff_self.1", c, c);
  k_lin(k, p + ".ff_self.3", c, c);
}

struct Topo {
  char kind;  // r(es) d(own) u(p) a(ttn)
  std::string name;
  int a, b;
};
static std::vector<Topo> unet_topo(int in_ch, bool deep) {
  std::vector<Topo> t = {{'r', "inc", in_ch, 64},   {'d', "down1", 64, 128}, {'a', "sa1", 128, 0},
                         {'d', "down2", 128, 256}, {'a', "sa2", 256, 0},    {'d', "down3", 256, 256},
                         {'a', "sa3", 256, 0}};
  if (deep) {
    t.push_back({'r', "bot1", 256, 512});
    t.push_back({'r', "bot2", 512, 512});
    t.push_back({'r', "bot3", 512, 256});
  } else {
    t.push_back({'r', "bot1", 256, 256});
    t.push_back({'r', "bot3", 256, 256});
  }
  std::vector<Topo> rest = {{'u', "up1", 512, 128}, {'a', "sa4", 128, 0}, {'u', "up2", 256, 64},
                            {'a', "sa5", 64, 0},    {'u', "up3", 128, 64}, {'a', "sa6", 64, 0}};
  t.insert(t.end(), rest.begin(), rest.end());
  return t;
}

// Constructor arguments of the reference networks that change the checkpoint layout.
struct ModelCfg {
  int kind = 0, in_ch = 4;
  bool deep = true;
  int ncls = 4;          // class_emb rows = num_classes + 1 (models/unet_cond.py:121)
  int gdim = 12, ghid = 256;  // GeomHead (models/unet_cond_geom.py:38-39,49)
  float scale = 0.18215f;     // VAE scale_factor (models/vae.py:11)
};

static Keys model_keys(const ModelCfg& c) {
  const int kind = c.kind, in_ch = c.in_ch;
  const bool deep = c.deep;
  Keys k;
  if (kind == DMX_VAE) {
    // models/vae.py:17-49
    const int enc[][4] = {{0, 3, 64, 3},    {3, 64, 64, 4},    {6, 64, 128, 3},
                          {9, 128, 128, 4}, {12, 128, 256, 3}, {15, 256, 256, 4}};
    for (auto& e : enc) {
      k.push_back({"enc." + std::to_string(e[0]) + ".weight", {e[2], e[1], e[3], e[3]}});
      k.push_back({"enc." + std::to_string(e[0]) + ".bias", {e[2]}});
      k.push_back({"enc." + std::to_string(e[0] + 1) + ".weight", {e[2]}});
      k.push_back({"enc." + std::to_string(e[0] + 1) + ".bias", {e[2]}});
    }
    k.push_back({"to_mu.weight", {4, 256, 1, 1}});
    k.push_back({"to_mu.bias", {4}});
    k.push_back({"to_logvar.weight", {4, 256, 1, 1}});
    k.push_back({"to_logvar.bias", {4}});
    const int dec[][5] = {{0, 4, 256, 3, 0},    {3, 256, 256, 4, 1}, {6, 256, 128, 3, 0},
                          {9, 128, 128, 4, 1},  {12, 128, 64, 3, 0}, {15, 64, 64, 4, 1}};
    for (auto& d : dec) {
      if (d[4]) k.push_back({"dec." + std::to_string(d[0]) + ".weight", {d[1], d[2], 4, 4}});
      else k.push_back({"dec." + std::to_string(d[0]) + ".weight", {d[2], d[1], d[3], d[3]}});
      k.push_back({"dec." + std::to_string(d[0]) + ".bias", {d[2]}});
      k.push_back({"dec." + std::to_string(d[0] + 1) + ".weight", {d[2]}});
      k.push_back({"dec." + std::to_string(d[0] + 1) + ".bias", {d[2]}});
    }
    k.push_back({"dec.18.weight", {3, 64, 3, 3}});
    k.push_back({"dec.18.bias", {3}});
    return k;
  }
  const bool cond = kind == DMX_UNET_COND_GEOM || kind == DMX_UNET_COND;
  if (cond) {
    k.push_back({"class_emb.weight", {c.ncls, 256}});
    k_lin(k, "cond_mlp.0", 24, 256);
    k_lin(k, "cond_mlp.2", 256, 256);
  }
  for (auto& t : unet_topo(in_ch, deep)) {
    if (t.kind == 'r') k_res(k, t.name, t.a, t.b);
    else if (t.kind == 'd') {
      k_res(k, t.name + ".maxpool_conv.1", t.a, t.a);
      k_res(k, t.name + ".maxpool_conv.2", t.a, t.b);
      k_lin(k, t.name + ".emb_layer.1", 256, t.b);
    } else if (t.kind == 'u') {
      k_res(k, t.name + ".conv.0", t.a, t.a);
      k_res(k, t.name + ".conv.1", t.a, t.b, t.a / 2);
      k_lin(k, t.name + ".emb_layer.1", 256, t.b);
    } else {
      k_attn(k, t.name, t.a);
    }
  }
  k.push_back({"out.weight", {in_ch, 64, 1, 1}});
  k.push_back({"out.bias", {in_ch}});
  if (kind == DMX_UNET_COND_GEOM) {
    k_lin(k, "geom_head.mlp.0", 64, c.ghid);
    k_lin(k, "geom_head.mlp.2", c.ghid, c.gdim);
  }
  return k;
}

// ===========================================================================
// Packed weights
// ===========================================================================
struct ConvW {
  float* B = nullptr;           // fp32 [phases][npad][kpad]
  _Float16* Bh = nullptr;       // split-precision planes (scaled by 1/inv_scale)
  _Float16* Bl = nullptr;
  _Float16* Fh = nullptr;       // the planes again in MFMA-fragment order (3x3 convs read by the
  _Float16* Fl = nullptr;       // halo kernel straight into registers; igemm_halo.h frag_planes_kernel)
  _Float16* Uh = nullptr;       // 3x3 convs: Winograd F(2x2, 3x3) weights U = G g Gᵀ, split, fragment
  _Float16* Ul = nullptr;       // order (igemm_wino.h wino_pack_kernel), same 2^e scale as Bh / Bl
  float inv_scale = 1.f;
  float* inv_dev = nullptr;     // device-side 2^-e of Bh / Bl (training data-gradient weights), or null
  unsigned* amax_dev = nullptr; //   and the max|B| slot it comes from
  float* bias = nullptr;
  int cin = 0, cout = 0, taps = 0, kpad = 0, npad = 0, phases = 1;
};
struct Vec {
  float* p = nullptr;
};
struct ResW {
  ConvW c1, c2;
  Vec g1, b1, g2, b2;
  int cin = 0, mid = 0, cout = 0;
  int cin_real = 0;     // channels of the reference tensor (cin is padded to a multiple of 4)
  std::string prefix;   // state_dict prefix ("down1.maxpool_conv.1")
  ConvW d1, d2;         // training: data-gradient GEMMs (flipped, transposed kernels; train.h)
  ConvW t1, t2;         // training forward: c1 / c2 with device-split f16 planes (or no planes: fp32)
};
struct AttnW {
  ConvW qkv, o, f1, f2;
  Vec l1w, l1b, l2w, l2b;
  int c = 0;
  std::string prefix;
  ConvW dqkv, dout, df1, df2;  // training: transposed Linear weights (data gradients)
  ConvW tqkv, to, tf1, tf2;    // training forward: device-split planes of qkv / o / f1 / f2
};
struct DownUpW {
  ResW r0, r1;
  int emb_off = 0, cout = 0;
};

// Workspace: bump allocator run twice (plan: sizes only, then real).
struct Arena {
  char* base = nullptr;
  size_t cap = 0, off = 0;
  bool plan = true;
  // DMX_CHECK: allocation sizes of the plan pass, compared one by one in the real pass
  std::vector<size_t>* trace = nullptr;
  size_t n = 0;
  const std::string* layer = nullptr;
  template <typename T>
  T* get(size_t count) {
    const size_t bytes = (count * sizeof(T) + 255) & ~(size_t)255;
    if (trace != nullptr) {
      if (plan) {
        trace->push_back(bytes);
      } else if (n >= trace->size() || (*trace)[n] != bytes) {
        throw std::runtime_error("workspace allocation " + std::to_string(n) + " differs between plan and run (" +
                                 std::to_string(n < trace->size() ? (*trace)[n] : 0) + " vs " +
                                 std::to_string(bytes) + " bytes, layer '" + (layer ? *layer : std::string()) + "')");
      }
      ++n;
    }
    char* p = base + off;
    off += bytes;
    // plan pass: a non-null placeholder, so code that tests a buffer pointer for null takes the
    // same branch (and allocates the same) in both passes; it is never dereferenced
    return reinterpret_cast<T*>(plan ? reinterpret_cast<char*>(static_cast<uintptr_t>(4096) + off) : p);
  }
};

struct GraphKey {
  dmx_step_args a;
  int table_gen;  // dmx_ctx::table_gen at capture
  bool operator==(const GraphKey& o) const { return std::memcmp(this, &o, sizeof(GraphKey)) == 0; }
};

struct Tape;  // training forward record (train_engine.h)

}  // namespace dmx

struct dmx_ctx {
  int device = 0;
  float* pos_table = nullptr;
  int tmax = 0;
  int table_gen = 0;  // bumped whenever pos_table is reallocated (captured graphs hold the old pointer)
};

struct dmx_model {
  dmx_ctx* ctx = nullptr;
  int kind = 0, in_ch = 4;
  bool deep = true;
  dmx::ModelCfg cfg;
  bool finalized = false;
  dmx::Keys keys;
  std::map<std::string, std::pair<const float*, std::vector<int64_t>>> inputs;
  std::vector<void*> owned;
  std::map<const char*, size_t> owned_bytes;  // DMX_CHECK operand-range validation
  // U-Net
  dmx::ResW inc, bot[3];
  int nbot = 0;
  dmx::DownUpW down[3], up[3];
  dmx::AttnW sa[6];
  float *class_emb = nullptr, *w0 = nullptr, *b0 = nullptr, *w2t = nullptr, *b2 = nullptr, *wht = nullptr,
        *bh = nullptr;
  int hsum = 0;
  float *out_w = nullptr, *out_b = nullptr, *gw0 = nullptr, *gb0 = nullptr, *gw2 = nullptr, *gb2 = nullptr;
  // VAE decoder
  dmx::ConvW vconv[4], vconvt[3];
  dmx::Vec vg[6], vb[6];
  // VAE encoder (conv3x3 / conv4x4-s2 implicit GEMMs, GN(8) affine, 1x1 heads as raw fp32)
  dmx::ConvW venc[6];
  dmx::Vec veg[6], veb[6];
  float *wmu = nullptr, *bmu = nullptr, *wlv = nullptr, *blv = nullptr;
  // workspace + graph
  dmx::Arena ws;
  void* ws_mem = nullptr;
  size_t ws_cap = 0;
  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  hipGraphExec_t gexec_k = nullptr;  // the same step captured kGraphSteps times back to back
  hipGraph_t graph_k = nullptr;
  dmx::GraphKey gkey{};
  bool has_graph = false;
  // debug taps: (name, device pointer into the workspace, element count, C)
  bool debug = false;
  int prec = 1;  // 0: fp32 MFMA (exact fp32 products), 1: fp16 hi/lo x3 split MFMA, 2: fp16 (config 4)
  int* range_flag = nullptr;  // device int: an output went non-finite (kernels.h flag_nonfinite)
  int64_t* t_scratch = nullptr;  // device int64: the 8-step graph's second t scalar (own allocation)

  std::vector<std::pair<std::string, std::pair<const float*, size_t>>> taps;
  // Weight packing replay (dmx_model_refresh): every device-side repack / copy of the caller's
  // tensors, in finalize order; the f16 planes of the split GEMMs are re-derived lazily
  // (planes_stale) before the next split-precision launch.
  std::vector<std::function<void(hipStream_t)>> jobs;
  std::vector<dmx::SplitJob> split_jobs;  // device-side splits of the training data-gradient weights,
  void* split_table = nullptr;            // replayed batched after the repacks (two launches)
  size_t split_table_n = 0, split_chunks = 0;
  std::vector<dmx::CopyJob> copies;     // parameter copies and weight repacks, replayed batched
  std::vector<dmx::RepackJob> repacks;  // (one launch each) by dmx_model_refresh
  void* job_tables = nullptr;           // device copies of the two tables
  size_t job_tables_n = 0;              // copies.size() + repacks.size() when uploaded
  size_t copy_chunks = 0, repack_chunks = 0, repack_tiles = 0;  // BatchChunk / RepackTile entries (kernels.h)
  bool planes_stale = false;
  unsigned* amax = nullptr;  // absmax scratch of split_planes
  // training (train_engine.h): tape of the last dmx_train_forward, its workspace and the
  // backward pass's workspace
  bool train_ready = false;
  dmx::Tape* tape = nullptr;
  dmx::Arena tws, bws;
  void *tws_mem = nullptr, *bws_mem = nullptr;
  size_t tws_cap = 0, bws_cap = 0;
  int64_t tape_id = 0;
};

namespace dmx {

// ---------------------------------------------------------------------------
// weight packing helpers (device-side repack of the caller's tensors)
// ---------------------------------------------------------------------------
// fp16 hi/lo planes of a packed fp32 B into c.Bh / c.Bl, scaled by 2^e so that
// max|w| * 2^e ~ 2^13 (one host read of the absmax).
static void split_planes(ConvW& c, hipStream_t st, unsigned* slot) {
  const size_t n = (size_t)c.phases * c.npad * c.kpad;
  HIPCHK(hipMemsetAsync(slot, 0, sizeof(unsigned), st));
  absmax_kernel<<<256, 256, 0, st>>>(c.B, n, slot);
  HIPCHK(hipGetLastError());
  unsigned bits = 0;
  HIPCHK(hipMemcpyAsync(&bits, slot, sizeof(unsigned), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  float mx;
  std::memcpy(&mx, &bits, sizeof(float));
  int e = 0;
  if (mx > 0.f && std::isfinite(mx)) e = std::max(-8, std::min(24, (int)std::floor(std::log2(8192.0f / mx))));
  const float scale = std::ldexp(1.0f, e);
  c.inv_scale = std::ldexp(1.0f, -e);
  split_weights_kernel<<<(int)std::min<size_t>((n + 255) / 256, 8192), 256, 0, st>>>(c.B, c.Bh, c.Bl, n, scale);
  HIPCHK(hipGetLastError());
  if (c.Fh != nullptr) {
    const size_t chunks = n / 8;
    frag_planes_kernel<<<(int)std::min<size_t>((chunks + 255) / 256, 8192), 256, 0, st>>>(c.Bh, c.Bl, c.Fh, c.Fl,
                                                                                          c.npad, c.kpad);
    HIPCHK(hipGetLastError());
  }
  if (c.Uh != nullptr) {  // max|U| <= 2.25 max|w|: the scaled U stays below 2^15 (f16-normal hi and lo)
    launch_wino_pack(c.B, c.kpad, c.cin, c.cout, scale, c.Uh, c.Ul, st);
    HIPCHK(hipGetLastError());
  }
}

// Every split-GEMM weight of the model (the f16 planes are re-derived after a refresh).
template <typename F>
static void for_each_conv(dmx_model* m, F&& f) {
  auto res = [&](ResW& r) {
    f(r.c1);
    f(r.c2);
  };
  res(m->inc);
  for (int i = 0; i < 3; ++i) {
    res(m->down[i].r0);
    res(m->down[i].r1);
    res(m->up[i].r0);
    res(m->up[i].r1);
    res(m->bot[i]);
  }
  for (auto& a : m->sa) {
    f(a.qkv);
    f(a.o);
    f(a.f1);
    f(a.f2);
  }
  for (auto& c : m->vconv) f(c);
  for (auto& c : m->vconvt) f(c);
  for (auto& c : m->venc) f(c);
}

struct Packer {
  dmx_model* m;
  hipStream_t st;
  const std::pair<const float*, std::vector<int64_t>>& in(const std::string& name) {
    auto it = m->inputs.find(name);
    if (it == m->inputs.end()) throw Error(DMX_E_STATE, "missing weight tensor '" + name + "'");
    return it->second;
  }
  float* alloc(size_t n) {
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, n * sizeof(float) + 256));
    m->owned.push_back(p);
    m->owned_bytes[static_cast<const char*>(p)] = n * sizeof(float) + 256;
    return static_cast<float*>(p);
  }
  // Run a packing step now and record it for dmx_model_refresh.
  void job(std::function<void(hipStream_t)> f) {
    f(st);
    m->jobs.push_back(std::move(f));
  }
  // f16 hi / lo planes of a packed fp32 B with a device-side scale (no host round trip), derived on
  // the device by run_split_jobs (the end of the training pack, and every refresh after the repacks):
  // the training data-gradient weights (train_engine.h)
  void split_dev(ConvW& c) {
    const size_t n = (size_t)c.phases * c.npad * c.kpad;
    void* h = nullptr;
    void* l = nullptr;
    void* a = nullptr;
    HIPCHK(hipMalloc(&h, n * sizeof(_Float16)));
    m->owned.push_back(h);
    HIPCHK(hipMalloc(&l, n * sizeof(_Float16)));
    m->owned.push_back(l);
    HIPCHK(hipMalloc(&a, SPLIT_PARTS * sizeof(unsigned) + 64));
    m->owned.push_back(a);
    c.Bh = static_cast<_Float16*>(h);
    c.Bl = static_cast<_Float16*>(l);
    c.amax_dev = static_cast<unsigned*>(a);
    c.inv_dev = reinterpret_cast<float*>(static_cast<char*>(a) + SPLIT_PARTS * sizeof(unsigned));
    m->split_jobs.push_back(SplitJob{c.B, c.Bh, c.Bl, c.amax_dev, c.inv_dev, n});
  }
  float* copy(const std::string& name) {
    auto& t = in(name);
    size_t n = 1;
    for (auto s : t.second) n *= (size_t)s;
    float* d = alloc(n);
    const float* src = t.first;
    HIPCHK(hipMemcpyAsync(d, src, n * sizeof(float), hipMemcpyDeviceToDevice, st));
    m->copies.push_back(CopyJob{d, src, n});  // replayed batched by dmx_model_refresh
    return d;
  }
  Vec vec(const std::string& name) { return Vec{copy(name)}; }
  // fp16 hi/lo planes of a packed fp32 B (split_planes below)
  void split(ConvW& c) {
    const size_t n = (size_t)c.phases * c.npad * c.kpad;
    void* h = nullptr;
    void* l = nullptr;
    HIPCHK(hipMalloc(&h, n * sizeof(_Float16)));
    m->owned.push_back(h);
    HIPCHK(hipMalloc(&l, n * sizeof(_Float16)));
    m->owned.push_back(l);
    c.Bh = static_cast<_Float16*>(h);
    c.Bl = static_cast<_Float16*>(l);
    if ((c.taps == 9 && c.phases == 1 && c.cout % 64 == 0 && c.cin % 32 == 0 && c.kpad == 9 * c.cin) ||
        (c.taps == 1 && c.phases == 1)) {
      // halo-kernel candidate (gemm(): 3x3, Cout % 64, whole 32-channel chunks) or a Linear read
      // by the token kernels (tokmlp.h tok_gemm: one coalesced 1 KB load per B fragment)
      HIPCHK(hipMalloc(&h, n * sizeof(_Float16)));
      m->owned.push_back(h);
      HIPCHK(hipMalloc(&l, n * sizeof(_Float16)));
      m->owned.push_back(l);
      c.Fh = static_cast<_Float16*>(h);
      c.Fl = static_cast<_Float16*>(l);
      if (c.taps == 9 && c.cin % 16 == 0) {  // Winograd candidate (gemm(): wino_ok)
        const size_t nu = (size_t)16 * c.cout * c.cin;
        HIPCHK(hipMalloc(&h, nu * sizeof(_Float16)));
        m->owned.push_back(h);
        HIPCHK(hipMalloc(&l, nu * sizeof(_Float16)));
        m->owned.push_back(l);
        c.Uh = static_cast<_Float16*>(h);
        c.Ul = static_cast<_Float16*>(l);
        m->owned_bytes[static_cast<const char*>(h)] = nu * sizeof(_Float16);  // DMX_CHECK ranges
        m->owned_bytes[static_cast<const char*>(l)] = nu * sizeof(_Float16);
      }
    }
    split_planes(c, st, absmax_slot());
  }
  unsigned* absmax_slot() {
    if (m->amax == nullptr) {
      void* d = nullptr;
      HIPCHK(hipMalloc(&d, 256));
      m->owned.push_back(d);
      m->amax = static_cast<unsigned*>(d);
    }
    return m->amax;
  }
  void repack(float* dst, const float* src, int kind, int P, int npad, int kpad, int cout, int cin, int ks) {
    const size_t total = (size_t)P * npad * kpad;
    const int blocks = (int)std::min<size_t>((total + 255) / 256, 8192);
    repack_kernel<<<blocks, 256, 0, st>>>(dst, src, kind, P, npad, kpad, cout, cin, ks);
    HIPCHK(hipGetLastError());
    // replayed batched by dmx_model_refresh, after the recorded jobs (which produce the
    // padded / flipped / transposed sources some repacks read)
    m->repacks.push_back(RepackJob{dst, src, kind, P, npad, kpad, cout, cin, ks});
  }
  // Conv2d [cout][cin][ks][ks]; channel-padded to cin_pad (in_ch=3 first layer)
  ConvW conv(const std::string& w, const std::string& b, int cin, int cout, int ks, int cin_pad = 0) {
    ConvW c;
    cin_pad = cin_pad ? cin_pad : cin;
    c.cin = cin_pad;
    c.cout = cout;
    c.taps = ks * ks;
    c.kpad = rup(c.taps * cin_pad, 64);
    c.npad = rup(cout, 128);
    c.B = alloc((size_t)c.npad * c.kpad);
    if (cin_pad == cin) {
      repack(c.B, in(w).first, 0, 1, c.npad, c.kpad, cout, cin, ks);
    } else {
      // pad input channels: repack into a temporary [cout][cin_pad][ks][ks] first
      float* tmp = alloc((size_t)cout * cin_pad * ks * ks);
      const float* src = in(w).first;
      job([=](hipStream_t s) {  // [cout][cin][k][k] rows into [cout][cin_pad][k][k] (zero padded)
        HIPCHK(hipMemsetAsync(tmp, 0, (size_t)cout * cin_pad * ks * ks * sizeof(float), s));
        HIPCHK(hipMemcpy2DAsync(tmp, (size_t)cin_pad * ks * ks * sizeof(float), src, (size_t)cin * ks * ks * sizeof(float),
                                (size_t)cin * ks * ks * sizeof(float), cout, hipMemcpyDeviceToDevice, s));
      });
      repack(c.B, tmp, 0, 1, c.npad, c.kpad, cout, cin_pad, ks);
    }
    if (!b.empty()) c.bias = copy(b);
    split(c);
    return c;
  }
  ConvW linear(const std::string& w, const std::string& b, int fin, int fout) {
    ConvW c;
    c.cin = fin;
    c.cout = fout;
    c.taps = 1;
    c.kpad = rup(fin, 64);
    c.npad = rup(fout, 128);
    c.B = alloc((size_t)c.npad * c.kpad);
    repack(c.B, in(w).first, 1, 1, c.npad, c.kpad, fout, fin, 1);
    c.bias = copy(b);
    split(c);
    return c;
  }
  ConvW convt(const std::string& w, const std::string& b, int cin, int cout) {
    ConvW c;
    c.cin = cin;
    c.cout = cout;
    c.taps = 4;
    c.phases = 4;
    c.kpad = rup(4 * cin, 64);
    c.npad = rup(cout, 128);
    c.B = alloc((size_t)4 * c.npad * c.kpad);
    repack(c.B, in(w).first, 2, 4, c.npad, c.kpad, cout, cin, 4);
    c.bias = copy(b);
    split(c);
    return c;
  }
  ResW res(const std::string& p, int cin, int cout, int mid = 0, int cin_pad = 0) {
    ResW r;
    mid = mid ? mid : cout;
    r.cin = cin_pad ? cin_pad : cin;
    r.mid = mid;
    r.cout = cout;
    r.cin_real = cin;
    r.prefix = p;
    r.c1 = conv(p + ".double_conv.0.weight", "", cin, mid, 3, cin_pad);
    r.g1 = vec(p + ".double_conv.1.weight");
    r.b1 = vec(p + ".double_conv.1.bias");
    r.c2 = conv(p + ".double_conv.3.weight", "", mid, cout, 3);
    r.g2 = vec(p + ".double_conv.4.weight");
    r.b2 = vec(p + ".double_conv.4.bias");
    return r;
  }
  AttnW attn(const std::string& p, int c) {
    AttnW a;
    a.c = c;
    a.prefix = p;
    a.qkv = linear(p + ".mha.in_proj_weight", p + ".mha.in_proj_bias", c, 3 * c);
    a.o = linear(p + ".mha.out_proj.weight", p + ".mha.out_proj.bias", c, c);
    a.l1w = vec(p + ".ln.weight");
    a.l1b = vec(p + ".ln.bias");
    a.l2w = vec(p + ".ff_self.0.weight");
    a.l2b = vec(p + ".ff_self.0.bias");
    a.f1 = linear(p + ".ff_self.1.weight", p + ".ff_self.1.bias", c, c);
    a.f2 = linear(p + ".ff_self.3.weight", p + ".ff_self.3.bias", c, c);
    return a;
  }
  float* transposed(const std::string& name, int rows, int cols) {
    float* d = alloc((size_t)rows * cols);
    const float* src = in(name).first;
    job([=](hipStream_t s) {
      transpose_kernel<<<std::min(cdiv(rows * cols, 256), 4096), 256, 0, s>>>(d, src, rows, cols);
      HIPCHK(hipGetLastError());
    });
    return d;
  }
};

static void finalize_model(dmx_model* m, hipStream_t st) {
  for (auto& k : m->keys) {
    auto it = m->inputs.find(k.name);
    if (it == m->inputs.end()) throw Error(DMX_E_STATE, "missing weight tensor '" + k.name + "'");
    if (it->second.second != k.shape) throw Error(DMX_E_ARG, "shape mismatch for '" + k.name + "'");
  }
  Packer P{m, st};
  if (m->kind == DMX_VAE) {
    m->vconv[0] = P.conv("dec.0.weight", "dec.0.bias", 4, 256, 3);
    m->vconvt[0] = P.convt("dec.3.weight", "dec.3.bias", 256, 256);
    m->vconv[1] = P.conv("dec.6.weight", "dec.6.bias", 256, 128, 3);
    m->vconvt[1] = P.convt("dec.9.weight", "dec.9.bias", 128, 128);
    m->vconv[2] = P.conv("dec.12.weight", "dec.12.bias", 128, 64, 3);
    m->vconvt[2] = P.convt("dec.15.weight", "dec.15.bias", 64, 64);
    const int gi[6] = {1, 4, 7, 10, 13, 16};
    for (int i = 0; i < 6; ++i) {
      m->vg[i] = P.vec("dec." + std::to_string(gi[i]) + ".weight");
      m->vb[i] = P.vec("dec." + std::to_string(gi[i]) + ".bias");
    }
    m->vconv[3].B = P.copy("dec.18.weight");
    m->vconv[3].bias = P.copy("dec.18.bias");
    // encoder (models/vae.py:17-30): conv3x3 s1 and conv4x4 s2 alternating, GN(8) + GELU after each
    const int eci[6] = {3, 64, 64, 128, 128, 256}, eco[6] = {64, 64, 128, 128, 256, 256};
    for (int i = 0; i < 6; ++i) {
      const std::string w = "enc." + std::to_string(3 * i);
      m->venc[i] = P.conv(w + ".weight", w + ".bias", eci[i], eco[i], (i & 1) ? 4 : 3, i == 0 ? 4 : 0);
      m->veg[i] = P.vec("enc." + std::to_string(3 * i + 1) + ".weight");
      m->veb[i] = P.vec("enc." + std::to_string(3 * i + 1) + ".bias");
    }
    m->wmu = P.copy("to_mu.weight");
    m->bmu = P.copy("to_mu.bias");
    m->wlv = P.copy("to_logvar.weight");
    m->blv = P.copy("to_logvar.bias");
  } else {
    const bool cond = m->kind != DMX_UNET;
    const int cin_pad = rup(m->in_ch, 4);
    m->inc = P.res("inc", m->in_ch, 64, 0, cin_pad);
    const char* dn[3] = {"down1", "down2", "down3"};
    const int dci[3] = {64, 128, 256}, dco[3] = {128, 256, 256};
    const char* un[3] = {"up1", "up2", "up3"};
    const int uci[3] = {512, 256, 128}, uco[3] = {128, 64, 64};
    int off = 0;
    for (int i = 0; i < 3; ++i) {
      m->down[i].r0 = P.res(std::string(dn[i]) + ".maxpool_conv.1", dci[i], dci[i]);
      m->down[i].r1 = P.res(std::string(dn[i]) + ".maxpool_conv.2", dci[i], dco[i]);
      m->down[i].emb_off = off;
      m->down[i].cout = dco[i];
      off += dco[i];
    }
    for (int i = 0; i < 3; ++i) {
      m->up[i].r0 = P.res(std::string(un[i]) + ".conv.0", uci[i], uci[i]);
      m->up[i].r1 = P.res(std::string(un[i]) + ".conv.1", uci[i], uco[i], uci[i] / 2);
      m->up[i].emb_off = off;
      m->up[i].cout = uco[i];
      off += uco[i];
    }
    m->hsum = off;
    if (m->deep) {
      m->bot[0] = P.res("bot1", 256, 512);
      m->bot[1] = P.res("bot2", 512, 512);
      m->bot[2] = P.res("bot3", 512, 256);
      m->nbot = 3;
    } else {
      m->bot[0] = P.res("bot1", 256, 256);
      m->bot[1] = P.res("bot3", 256, 256);
      m->nbot = 2;
    }
    const int sac[6] = {128, 256, 256, 128, 64, 64};
    for (int i = 0; i < 6; ++i) m->sa[i] = P.attn("sa" + std::to_string(i + 1), sac[i]);
    // embedding heads: transposed & concatenated [256][hsum]
    m->wht = P.alloc((size_t)256 * m->hsum);
    m->bh = P.alloc(m->hsum);
    const char* all[6] = {"down1", "down2", "down3", "up1", "up2", "up3"};
    const int hc[6] = {128, 256, 256, 128, 64, 64};
    int o = 0;
    for (int i = 0; i < 6; ++i) {
      float* tp = P.transposed(std::string(all[i]) + ".emb_layer.1.weight", hc[i], 256);  // [256][hc]
      float* wd = m->wht + o;
      float* bd = m->bh + o;
      const float* bs = P.in(std::string(all[i]) + ".emb_layer.1.bias").first;
      const int hs = m->hsum, w = hc[i];
      P.job([=](hipStream_t s) {
        HIPCHK(hipMemcpy2DAsync(wd, (size_t)hs * sizeof(float), tp, (size_t)w * sizeof(float), (size_t)w * sizeof(float),
                                256, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(bd, bs, w * sizeof(float), hipMemcpyDeviceToDevice, s));
      });
      o += hc[i];
    }
    if (cond) {
      m->class_emb = P.copy("class_emb.weight");
      m->w0 = P.copy("cond_mlp.0.weight");
      m->b0 = P.copy("cond_mlp.0.bias");
      m->w2t = P.transposed("cond_mlp.2.weight", 256, 256);
      m->b2 = P.copy("cond_mlp.2.bias");
    }
    m->out_w = P.copy("out.weight");
    m->out_b = P.copy("out.bias");
    if (m->kind == DMX_UNET_COND_GEOM) {
      m->gw0 = P.copy("geom_head.mlp.0.weight");
      m->gb0 = P.copy("geom_head.mlp.0.bias");
      m->gw2 = P.copy("geom_head.mlp.2.weight");
      m->gb2 = P.copy("geom_head.mlp.2.bias");
    }
  }
  {
    void* f = nullptr;
    HIPCHK(hipMalloc(&f, 256));
    m->owned.push_back(f);
    m->range_flag = static_cast<int*>(f);
    HIPCHK(hipMemsetAsync(f, 0, 256, st));
    void* t = nullptr;
    HIPCHK(hipMalloc(&t, 256));
    m->owned.push_back(t);
    m->t_scratch = static_cast<int64_t*>(t);
    HIPCHK(hipMemsetAsync(t, 0, 256, st));
  }
  HIPCHK(hipStreamSynchronize(st));
  // the registered tensors stay referenced only by dmx_model_refresh / training (include/dmx.h)
  m->finalized = true;
}

// ===========================================================================
// Launch helpers
// ===========================================================================
struct ProfRec {
  std::string kernel, layer;
  double flops, bytes;
  hipEvent_t e0, e1;
};
struct Prof {
  std::vector<ProfRec> recs;
  std::vector<hipEvent_t> pool;
  hipEvent_t ev() {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    pool.push_back(e);
    return e;
  }
  ~Prof() {
    for (auto e : pool) (void)hipEventDestroy(e);
  }
};

// DMX_CKSUM=1 (diagnostic, eager dmx_step / dmx_unet_forward only): the workspace is filled with
// 0xFF before the step and, at the end of every layer, a 64-bit weighted sum of its used part is
// recorded; at the end of the step the sums are compared with the previous step's and the first
// layer after which they differ is printed (a race localiser: identical inputs must give identical
// sums).
// Diagnostic builds only (-DDMX_DIAG=1, e.g. `build.py --out libdiag.so -- -DDMX_DIAG=1`): product
// builds take no such switch.
#ifndef DMX_DIAG
#define DMX_DIAG 0
#endif
static bool cksum_enabled() {
#if DMX_DIAG
  static const bool v = [] {
    const char* e = std::getenv("DMX_CKSUM");
    return e != nullptr && std::atoi(e) != 0;
  }();
  return v;
#else
  return false;
#endif
}
static __global__ void cksum_kernel(const unsigned* p, size_t n, unsigned long long* slot) {
  unsigned long long s = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += p[i] * (i | 1);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(slot, s);
}
struct Cksum {
  unsigned long long* dev = nullptr;
  std::vector<std::string> names, prev_names;
  std::vector<unsigned long long> prev;
  int runs = 0;
};
static Cksum& cksum_state() {
  static Cksum c;
  return c;
}

struct Run {
  dmx_model* m;
  hipStream_t st;
  bool plan;
  Arena& ws;
  Prof* prof = nullptr;
  std::string layer;
  // > 0: gemm() takes its tile / split-K / kernel decisions as if the batch had this many
  // samples (the grid still covers the real batch).  The VAE decoder sets 1, so a sample's
  // decoded bytes do not depend on the batch or chunk it is decoded in (summation order is a
  // function of the per-sample geometry only).
  int tile_n = 0;
  // non-null: the next gemm() runs the split-precision implicit GEMM with A scaled on the device by
  // this max|A| slot (training data gradients, train_engine.h dgrad)
  bool fwd_x3 = false;  // training forward: weights with device-split planes (ConvW::inv_dev) run the split GEMM
  bool colsum_defer = false;               // training backward: final-level column sums batched (train_engine.h)
  std::vector<ColsumJob> colsums;
  const unsigned* a_amax = nullptr;
  int a_nparts = 0;  // a_amax: that many per-block partial maxima (absmax_part_kernel)
  // train_engine.h dy_amax: the last tensor whose |max| partials were taken
  const float* amax_src = nullptr;
  size_t amax_n = 0;
  unsigned* amax_slot = nullptr;
  int amax_parts = 0;
  int amax_uses = 0;  // remaining reuses of that measurement
  void tap(const std::string& name, const float* p, size_t count);
  std::string ck_layer;
  // DMX_CKSUM: one workspace checksum per layer, taken when the next layer's first kernel begins
  // set by run_planned's real pass only: graph captures (dmx_sample_loop, dmx_step_profile) build
  // their own Runs and never take checksums (the device slots may not exist yet, and a captured
  // atomic would replay into stale slots)
  bool cksum = false;
  void ck() {
    Cksum& c = cksum_state();
    if (!cksum || plan || c.dev == nullptr || m->ws_mem == nullptr || ck_layer.empty() || c.names.size() >= 1024)
      return;
    cksum_kernel<<<1024, 256, 0, st>>>(static_cast<const unsigned*>(m->ws_mem), ws.off / 4, c.dev + c.names.size());
    c.names.push_back(ck_layer);
  }
  void begin(const std::string& kernel, double flops, double bytes) {
    if (cksum && layer != ck_layer) {
      ck();
      ck_layer = layer;
    }
    if (!prof) return;
    ProfRec r{kernel, layer, flops, bytes, prof->ev(), prof->ev()};
    HIPCHK(hipEventRecord(r.e0, st));
    prof->recs.push_back(r);
  }
  void end() {
    if (!prof) return;
    HIPCHK(hipEventRecord(prof->recs.back().e1, st));
  }
};

void Run::tap(const std::string& name, const float* p, size_t count) {
  if (plan || !m->debug) return;
  m->taps.push_back({name, {p, count}});
}

// Mid-ResBlock activation emitted as fp16 hi/lo planes for the split GEMM.
static bool split_a_enabled() { return true; }

// Max-pool / up-concat sources also written as f16 planes for the next conv1 (split GEMM A;
// measured +0.2 %, same-box A/B) — they stay fp32 too, as the residual of that ResBlock.
// Planes are skipped where conv1 runs a halo / Winograd conv, which splits an fp32 source while
// staging — the source is written once (fp32, also the block's residual) instead of twice:
// prep_kernel<3> at 32 x 32 41.5 -> 32.9 us, the convs unchanged, +1.3 % per CFG step over planes
// for every source (same-box A/B, round 3; the switch was removed in round 6).
static bool cat_planes_enabled() { return true; }

// The 512-thread ping-pong kernel for the large f16-plane convs (measured +1.3 % over the
// two-block kernel, same-box A/B).
static bool pp_enabled() { return true; }

// The halo-staged 3x3 conv (igemm_halo.h) for the large 16x16 / 32x32 convs (the small-batch class;
// batches of >= 64 samples run Winograd): B staged in LDS per step, 16-wave blocks (4 x 4 waves of
// 64 x 32 at BN = 128, 8 x 2 of 32 x 32 at BN = 64) — +2.1 % per CFG step over 8-wave blocks, which
// were +2.4 … +2.7 % over the ping-pong / register-staged kernels it replaced (round 3 A/Bs; the
// losing layouts were removed in round 6).
constexpr int HALO_MODE = 4;
static bool halo_enabled() { return true; }
// Grids with fewer blocks than this split K: 256 (one block per CU).  Since the low-resolution convs
// moved to the halo kernels (own split rule), this only decides the implicit GEMMs of small
// batches; unsplit 256-block grids run their GroupNorm as norm_kernel over many blocks instead of
// reduce_norm_kernel's one block per sample (+0.25 % per CFG step over 512, 3/3 same-box rounds).
static int split_below() { return 256; }
// reduce_norm_kernel runs with at least two float4 per thread (KV >= 2; the 4x4 C = 256 ResBlocks,
// 1024 float4 per sample, leave the second one idle).  The one-float4 instance (KV = 1) gave
// run-to-run different outputs while a second process shared the GPU (tools/conc_step.sh +
// DMX_CKSUM: first difference after down3.0 / down3.1 / bot3, its three users), the KV = 2 instance
// on the same data never did (0 of 72).  The round-5 ISA review found no mechanism in the kernel
// (no scratch, lgkmcnt(0) before both barriers, st_s read behind the second barrier, no
// scalar loads of data, the producer covers every slab element — DMX_POISON), so the instance is not
// compiled at all: no knob can select it.
constexpr int RN_MIN_KV = 2;
// Split-K slabs of a ResBlock conv go straight into reduce_norm_kernel (slab sum + GroupNorm in one
// launch), and the mid-ResBlock GroupNorm + GELU is folded into conv2's staging where that pays
// (DMX_RN_FUSE / DMX_GN_FUSE A/B and bisection switches until round 5: always on since).
static bool rn_fuse_enabled() { return true; }
static bool gn_fuse_enabled() { return true; }

// Implicit GEMM: conv3x3 (taps 9), ConvT phases (taps 4, phases 4), conv4x4-s2 (taps 16),
// linear (taps 1).  Sources are plain NHWC (or the NCHW network input); grids too small to
// fill the 256 CUs are split along K into deterministic slabs reduced by splitk_reduce_kernel
// (or, in a ResBlock, by the caller's fused reduce_norm_kernel).
// Returns the GroupNorm partial rows per sample it wrote (EPI_STATS).
struct Deferred {
  bool fused = false;
  float* partial = nullptr;
  int splits = 0;
  const float* bias = nullptr;
};

// Diagnostic (DMX_CHECK=1): before every implicit-GEMM launch, verify that each operand range
// lies inside one allocation the model owns (packed weights, workspaces) and throw otherwise —
// an out-of-range operand is reported on the host instead of faulting the GPU.
static bool check_args() {
  static const bool v = [] {
    const char* e = std::getenv("DMX_CHECK");
    return e != nullptr && std::atoi(e) != 0;
  }();
  return v;
}
static void check_range(Run& R, const void* p, size_t bytes, const char* what) {
  if (!check_args() || p == nullptr || bytes == 0) return;
  const char* a = static_cast<const char*>(p);
  const dmx_model* m = R.m;
  auto inside = [&](const void* base, size_t cap) {
    const char* b = static_cast<const char*>(base);
    return base != nullptr && a >= b && a + bytes <= b + cap;
  };
  if (inside(m->ws_mem, m->ws_cap) || inside(m->tws_mem, m->tws_cap) || inside(m->bws_mem, m->bws_cap)) return;
  auto it = m->owned_bytes.upper_bound(a);
  if (it != m->owned_bytes.begin()) {
    --it;
    if (a >= it->first && a + bytes <= it->first + it->second) return;
  }
  char msg[512];
  std::snprintf(msg, sizeof msg,
                "DMX_CHECK: %s operand [%p, +%zu) of layer '%s' lies outside every model allocation "
                "(ws %p +%zu, tws %p +%zu, bws %p +%zu, arena off %zu)",
                what, p, bytes, R.layer.c_str(), m->ws_mem, m->ws_cap, m->tws_mem, m->tws_cap, m->bws_mem, m->bws_cap,
                R.ws.off);
  throw Error(DMX_E_INTERNAL, msg);
}

// GroupNorm(1, C) + GELU applied by the halo conv while it stages its raw fp32 source (the
// ResBlock's mid normalisation, igemm_halo.h GNA).
struct GnLoad {
  const float2* rowpart = nullptr;  // [N][cnt] partials of the producing conv
  int cnt = 0;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  const float* res = nullptr;       // non-null: GELU(res + GroupNorm(x)) (residual ResBlock output)
};

// Batch the tiling / split-K decisions are taken for: the VAE decoder's per-sample tile (Run::tile_n);
// for the U-Net a batch class — 128 samples (the benchmark's CFG batch) for every batch of >= 64, so
// a config-3 shard of 64 samples per rank (128 with CFG) and the whole 128-sample batch (256) sum
// every output in the same order (bit-identical latents, test_gpu_multi.py); below 64 the batch itself
// (each kernel's partial-tile rules keep a small batch and its shards alike: test_gpu_poison.py).
// Trade-off: batches far above 128 samples — a single-process B = 512 CFG batch of 1024
// samples, a large training forward — take the split-K / Winograd-split / tile decisions of 128 samples
// although their grids would fill the chip unsplit: more launches of the reduce kernels and split slabs
// of splits * M * Cout floats (workspace linear in the batch, test_large_batch_class_is_shard_exact
// bounds it) instead of whole-K tiles.  A coarser class above 128 would put a 64-per-rank shard and its
// parent batch in different classes and lose config 3's bit-identical shards.
static int dec_n(const Run& R, int N) { return R.tile_n > 0 ? R.tile_n : N >= 64 ? 128 : N; }

// Output-channel tile of the halo-staged 3x3 conv for this GEMM, or 0 when it does not apply
// (igemm_halo.h: 256-pixel tiles of whole rows of one sample, W = 16 / 32, 32-channel chunks,
// >= 256 blocks without split-K, EPI_STATS).
static int halo_bn(const Run& R, int src_C, int N, int H, int W, const ConvW& cw, int epi, bool plain_or_planes) {
  const int Md = dec_n(R, N) * H * W;
  const bool x3 = R.m->prec >= 1 && cw.Bh != nullptr;
  if (!(halo_enabled() && x3 && epi == EPI_STATS && cw.phases == 1 && cw.taps == 9 && (W == 16 || W == 32) &&
        (H * W) % 256 == 0 && src_C % 32 == 0 && cw.kpad == 9 * src_C && cw.Fh != nullptr && plain_or_planes))
    return 0;
  if (cw.cout % 128 == 0 && (Md / 256) * (cw.cout / 128) >= 256) return 128;
  if (cw.cout % 64 == 0 && (Md / 256) * (cw.cout / 64) >= 256) return 64;
  return 0;
}

// Low-resolution halo conv (8 x 8 / 4 x 4, the small-batch class): the chunk-staged kernel
// (igemm_halo_cs_kernel) everywhere — +1.5 % per CFG step over implicit GEMM + split-K; the per-tap
// pipeline and mixed layouts measured in between (round 3 A/Bs; removed in round 6).
static bool halo_ms_enabled() { return true; }

// GELU form of the exact-fp32 mode (training forward, fp32 reference mode): the erf form, as the
// reference (the fit's own effect on the training gradients was measured at <= 7.8e-8).
static int gelu_exact_flag(const Run& R) { return R.m->prec == 0 ? 1 : 0; }

// The Winograd conv (x3 fp32-semantics and fp16 modes, fp32 source, 64-tile x 64-channel blocks,
// 16-channel chunks) replaces the halo convs for batches of >= 64 samples, with K split over 16-channel
// chunks where the 64 x 64 blocks do not fill 256 CUs (slabs reduced like the other split convs).
// (DMX_WINO / DMX_WINO_SPLIT / DMX_WINO_F16 / DMX_WINO_MASK A/B switches until round 5.)
// Winograd plan of a 3x3 conv given an fp32 source: 0 = not applicable, else the K split count
// (1 = whole K) and *cps = 16-channel chunks per split.  Blocks: 64 tiles (8 rows of a 32-wide map,
// one 16 x 16 sample, four 8 x 8 samples or sixteen 4 x 4 samples — the last block of a batch that
// is not a multiple of 4 / 16 holds fewer) x 64 output channels.  The split count is a function of the conv's shape and of a
// coarse batch class only: it is planned for a reference batch of 128 samples (the benchmark's CFG
// batch) when the batch has >= 64 samples, of 2 samples below that (single-sample and small batches
// keep a full grid).  A batch and its shards in the same class sum every output in the same order
// (bit-identical results: test_gpu_poison.py's B = 5 vs 3 + 2; a 64-per-rank shard plans as the bench).
// Winograd geometry of an H x W map (igemm_wino.h): the block width 32 / 16 / 8 / 4 the map fits —
// 8-row bands of any height at 32, whole samples (H <= width) below; 0 = none.  The reference's 28 x 28
// latents (diff.py:315-322) run their 28 / 14 / 7 / 3 maps in the 32 / 16 / 8 / 4 geometries.
static int wino_geom(int H, int W) {
  if (W > 16 && W <= 32) return 32;
  const int g = W > 8 ? 16 : W > 4 ? 8 : W >= 2 ? 4 : 0;
  return (g != 0 && H <= g) ? g : 0;
}
static int wino_blocks(int G, int N, int H) {  // blocks along the pixel axis
  return G == 32 ? N * cdiv(H, 8) : cdiv(N, G == 8 ? 4 : G == 4 ? 16 : 1);
}
static int wino_plan(const Run& R, int src_C, int N, int H, int W, const ConvW& cw, int* cps) {
  // (U-Net only: the VAE decoder keeps its per-sample-tiled direct convs, Run::tile_n)
  if (R.m->prec < 1 || R.m->kind == DMX_VAE ||
      R.tile_n > 0 || cw.Uh == nullptr ||
      cw.phases != 1 || cw.taps != 9)
    return 0;
  const int G = wino_geom(H, W);
  if (G == 0) return 0;
  if (src_C % 16 != 0 || cw.cout % 64 != 0 || (size_t)16 * cw.cout * src_C * 2 >= ((size_t)1 << 31)) return 0;
  const int nref = dec_n(R, N) >= 64 ? 128 : 2;
  const int blocks = wino_blocks(G, nref, H) * (cw.cout / 64), nch = src_C / 16;
  int sp = 1, cp = nch;
  if (blocks < 256) {
    // (small-batch class: the split Winograd conv lost to the direct kernels — config 5, B = 1 CFG:
    // 1.44 vs 1.31 ms per step, same box)
    if (nref < 128) return 0;
    sp = std::max(1, std::min(nch, cdiv(256, blocks)));
    cp = cdiv(nch, sp);
    sp = cdiv(nch, cp);
  }
  if (G == 4 && sp == 1) return 0;  // (4 x 4: split-K instances only; sixteen samples per block)
  if (cps != nullptr) *cps = cp;
  return sp;
}
static bool wino_any(const Run& R, int src_C, int N, int H, int W, const ConvW& cw) {
  return wino_plan(R, src_C, N, H, W, cw, nullptr) > 0;
}
// GroupNorm(-residual)-GELU on load into a Winograd conv is applied once per 64-channel output block,
// i.e. Cout / 64 times per staged element, on the VALU the input transform already loads (diagnostic
// build without it: -11 % per step).  Same-box per-conv A/B against a norm_kernel pass + plain
// staging: Cout = 64 GN + GELU fused wins (-8 us at 32x32, -6 us at 16x16 split), Cout = 128 even,
// Cout >= 256 and every GroupNorm-residual-GELU (which also reads the residual) lose 10-42 us.
// The 4-wide geometry has no GroupNorm-on-load instances (split-K only), so a conv on a map of width
// <= 4 never takes it (the launcher would throw mid-forward otherwise).
static bool wino_gna_pays(const ConvW& cw, int gna, int W) { return gna == 1 && cw.cout <= 64 && wino_geom(1, W) != 4; }

// Low-resolution halo conv (igemm_halo.h, W = 8 / 4 square maps): 256-pixel tiles of whole samples,
// K split over 32-channel chunks until the grid has >= 256 blocks.  Returns the output-channel tile
// (0: not applicable) and the split count / chunks per split.
static int halo_ms_bn(const Run& R, int src_C, int N, int H, int W, const ConvW& cw, int epi, bool plain_or_planes,
                      int* splits, int* cps) {
  const int Md = dec_n(R, N) * H * W;
  const bool x3 = R.m->prec >= 1 && cw.Bh != nullptr;
  if (!(halo_ms_enabled() && x3 && epi == EPI_STATS && cw.phases == 1 && cw.taps == 9 && H == W &&
        (W == 8 || W == 4) && src_C % 32 == 0 &&
        cw.kpad == 9 * src_C && plain_or_planes))
    return 0;
  // decisions from Md: a batch not a multiple of 256 / W² samples ends in a partial tile; small
  // batches all split K into every chunk (the same summation order for a batch and its shards)
  const int nch = src_C / 32, mt = cdiv(Md, 256);
  auto plan = [&](int bn, int& sp, int& cp) {
    const int tiles = mt * (cw.cout / bn);
    sp = std::max(1, std::min(nch, cdiv(256, tiles)));
    cp = cdiv(nch, sp);
    sp = cdiv(nch, cp);
    return tiles * sp;
  };
  int sp = 1, cp = nch, bn = 0;
  if (cw.cout % 64 == 0) {
    plan(64, sp, cp);
    bn = 64;
  }
  if (bn == 0 || (W == 4 && sp == 1)) return 0;  // W = 4: EPI_PARTIAL instances only
  *splits = sp;
  *cps = cp;
  return bn;
}

static bool halo_ms_bn_any(const Run& R, int src_C, int N, int H, int W, const ConvW& cw) {
  int sp = 0, cp = 0;
  return halo_ms_bn(R, src_C, N, H, W, cw, EPI_STATS, true, &sp, &cp) > 0;
}

static int gemm(Run& R, const SrcDesc& s, int src_mode, int N, int H, int W, const ConvW& cw, int epi, float* out,
                const float* res, float2* rowpart, int seg, const _Float16* ash = nullptr,
                const _Float16* asl = nullptr, Deferred* defer = nullptr, const GnLoad* gn = nullptr) {
  const int M = N * H * W;
  const int Md = dec_n(R, N) * H * W;  // rows the decisions below are taken for
  if (cw.cout % 32 != 0) throw Error(DMX_E_INTERNAL, "gemm: Cout must be a multiple of 32");
  const int cin_px = W % 32 == 0 ? 32 : (W >= 16 && W <= 32 && (H * W) % 16 == 0) ? 16 : 0;  // conv_in_kernel<PX>
  if (src_mode == SRC_NCHW && epi == EPI_STATS && cw.taps == 9 && cw.phases == 1 && cw.cin == 4 && cw.cout == 64 &&
      cin_px > 0 && seg == 32 && cw.bias == nullptr && R.m->kind != DMX_VAE && gn == nullptr) {
    // inc's first conv: direct fp32 conv of the NCHW input (kernels.h conv_in_kernel; 16-pixel blocks for
    // the 28-wide latents)
    if (res != nullptr) throw Error(DMX_E_INTERNAL, "gemm: the direct input conv takes no residual");
    if (ash != nullptr || asl != nullptr) throw Error(DMX_E_INTERNAL, "gemm: the direct input conv reads fp32 NCHW");
    if (defer != nullptr) *defer = Deferred{};  // whole K, no slabs
    if (R.plan) return H * W / cin_px;
    if (check_args()) {  // (as every other GEMM path; the NCHW input is the caller's tensor, not checked)
      check_range(R, cw.B, (size_t)cw.phases * cw.npad * cw.kpad * 4, "B");
      check_range(R, out, (size_t)M * 64 * 4, "out");
      check_range(R, rowpart, (size_t)N * (H * W / cin_px) * (64 / 32) * sizeof(float2), "rowpart");
    }
    ConvInParams q;
    q.x = s.src0;
    q.creal = s.C0 ? s.C0 : s.C;
    q.n_mod = s.n_mod;
    q.scale = s.scale;
    q.B = cw.B;
    q.cin = cw.cin;
    q.kpad = cw.kpad;
    q.out = out;
    q.rowpart = rowpart;
    q.H = H;
    q.W = W;
    R.begin(cin_px == 32 ? "conv_in_kernel<32>" : "conv_in_kernel<16>", 2.0 * M * 64.0 * 9.0 * q.creal,
            4.0 * ((double)M * 64 + (double)M * q.creal));
    if (cin_px == 32) conv_in_kernel<32><<<M / 32, 256, 0, R.st>>>(q);
    else conv_in_kernel<16><<<M / 16, 256, 0, R.st>>>(q);
    R.end();
    HIPCHK(hipGetLastError());
    return H * W / cin_px;
  }
  const int bn = (cw.cout % 128 == 0) ? 128 : 64;
  const int tiles128 = cdiv(Md, 128) * cdiv(cw.cout, bn) * cw.phases;
  const int bm = tiles128 >= 256 ? 128 : 64;  // 128-row tiles (split K if the grid is then small) from 256 tiles
  const int blocks = cdiv(Md, bm) * cdiv(cw.cout, bn) * cw.phases;
  // (R.a_amax: a training data gradient on the split GEMM with device-side operand scales; R.fwd_x3:
  // the training forward's weights with device-split planes — whatever the model's precision mode,
  // only the implicit-GEMM kernels below carry those scales)
  const bool x3 = (R.m->prec >= 1 || R.a_amax != nullptr || (R.fwd_x3 && cw.inv_dev != nullptr)) &&
                  src_mode == SRC_PLAIN && cw.Bh != nullptr;
  if (R.a_amax != nullptr && (!x3 || ash != nullptr || epi == EPI_STATS || gn != nullptr || R.m->prec == 2))
    throw Error(DMX_E_INTERNAL, "gemm: device-scaled operands only on the plain split implicit GEMM");
  const bool x1 = x3 && R.m->prec == 2;  // config-4 fp16: one MFMA on the hi planes
  // 512-thread ping-pong kernel (256-row tiles) for the large f16-plane convs
  const bool pp = pp_enabled() && x3 && epi == EPI_STATS && cw.phases == 1 && s.C >= 32 && ash != nullptr &&
                  (H * W) % 32 == 0 && cdiv(Md, 256) * cdiv(cw.cout, bn) >= 256;  // 32-row GN partials
  // halo-staged 3x3 conv (igemm_halo.h): 256-pixel tiles of whole image rows (W = 16 / 32), the
  // chunk's input halo staged once for all nine taps; where it fills >= 256 blocks without split-K
  const int hbn = halo_bn(R, s.C, N, H, W, cw, epi, ash != nullptr || src_mode == SRC_PLAIN);
  int wsp = 0, wcps = 0;
  if (epi == EPI_STATS && src_mode == SRC_PLAIN && ash == nullptr) wsp = wino_plan(R, s.C, N, H, W, cw, &wcps);
  const bool wino = wsp > 0;
  if (gn != nullptr && ((hbn == 0 && !wino) || ash != nullptr || src_mode != SRC_PLAIN))
    throw Error(DMX_E_INTERNAL, "gemm: GroupNorm-on-load needs the halo / Winograd conv on a plain fp32 source");
  int ms_splits = 1, ms_cps = 0;
  const int msbn = (hbn || wino) ? 0
                       : halo_ms_bn(R, s.C, N, H, W, cw, epi, ash != nullptr || src_mode == SRC_PLAIN, &ms_splits,
                                    &ms_cps);
  const int bk = pp ? 32 : x3 ? 64 : IG_BK;
  const int nkt = cw.kpad / bk;
  int splits = 1, ksplit = nkt;
  if (wino) {  // Winograd: K split over 16-channel chunks where 64 x 64 blocks do not fill the chip
    splits = wsp;
    ksplit = wcps;
  } else if (msbn) {  // low-resolution halo conv: K split over channel chunks (ksplit = chunks per split)
    splits = ms_splits;
    ksplit = ms_cps;
  } else if (!hbn && !wino && !pp && cw.phases == 1 && blocks < split_below() && nkt * bk >= 512) {  // split K below 2 blocks / CU
    splits = std::min(std::min(8, std::max(2, 512 / blocks)), nkt * bk / 256);
    ksplit = cdiv(nkt, splits);
    splits = cdiv(nkt, ksplit);
  }
  float* partial = splits > 1 ? R.ws.get<float>((size_t)splits * M * cw.cout) : nullptr;
  const int rgrp = (splits == 1 && (H * W) % 32 == 0) ? 32 : 1;
  const int wg = wino ? wino_geom(H, W) : 0;
  // GroupNorm partial rows / sample (Winograd: one per 4 tiles of the geometry, igemm_wino.h)
  const int rrows = (wino && splits == 1) ? wino_blocks(wg, 1, H) * 64 / (wg == 8 ? 4 : wg == 4 ? 16 : 1) / 4
                                          : cw.phases * H * W / rgrp;
  if (defer != nullptr) {
    defer->fused = splits > 1 && epi == EPI_STATS && !R.m->debug && rn_fuse_enabled() &&
                   H * W * (cw.cout / 4) <= RN_MAXV * 1024;  // (debug taps read the raw conv output)
    defer->partial = partial;
    defer->splits = splits;
    defer->bias = cw.bias;
  }
  if (R.plan) return rrows;
  IgemmParams p;
  std::memset(&p, 0, sizeof(p));
  p.src = s;
  p.H = H;
  p.W = W;
  p.M = M;
  p.taps = cw.taps;
  p.geom = cw.phases == 4 ? 2 : (cw.taps == 9 ? 1 : (cw.taps == 16 ? 3 : 0));
  p.Hin = p.geom == 3 ? 2 * H : H;  // geom 3 (4x4 / s2 conv): H x W is the output grid
  p.Win = p.geom == 3 ? 2 * W : W;
  p.Kreal = cw.taps * cw.cin;
  p.Kpad = cw.kpad;
  p.Cout = cw.cout;
  p.Npad = cw.npad;
  p.osy = p.osx = cw.phases == 4 ? 2 : 1;
  p.Hout = H * p.osy;
  p.Wout = W * p.osx;
  p.Bw = cw.B;
  p.bias = cw.bias;
  p.out = out;
  p.res = res;
  p.rowpart = rowpart;
  p.seg = seg;
  p.ksplit = ksplit;
  p.partial = partial;
  p.rgrp = rgrp;
  p.nphase = cw.phases;
  p.gexact = gelu_exact_flag(R);
  if (s.C != cw.cin) throw Error(DMX_E_INTERNAL, "gemm: source channels != weight channels");
  if (x3 && cw.cin < bk) throw Error(DMX_E_INTERNAL, "gemm: x3 path needs Cin >= K-step");
  if (ash != nullptr && !x3) throw Error(DMX_E_INTERNAL, "gemm: f16-plane operand needs the split GEMM");
  if (src_mode != SRC_PLAIN && src_mode != SRC_NCHW) throw Error(DMX_E_INTERNAL, "gemm: unsupported source");
  if (check_args()) {
    if (src_mode == SRC_PLAIN)
      check_range(R, s.src0, (size_t)N * p.Hin * p.Win * s.C * 4, "A");
    check_range(R, ash, (size_t)N * p.Hin * p.Win * s.C * 2, "A hi");
    check_range(R, asl, (size_t)N * p.Hin * p.Win * s.C * 2, "A lo");
    check_range(R, cw.B, (size_t)cw.phases * cw.npad * cw.kpad * 4, "B");
    check_range(R, partial, (size_t)splits * M * cw.cout * 4, "partial");
    if (!(splits > 1 && defer != nullptr && defer->fused))
      check_range(R, out, (size_t)N * p.Hout * p.Wout * cw.cout * 4, "out");
    check_range(R, res, (size_t)N * p.Hout * p.Wout * cw.cout * 4, "res");
  }
  X3Params xp;
  xp.g = p;
  xp.Ash = ash;
  xp.Asl = asl;
  xp.Bh = cw.Bh;
  xp.Bl = cw.Bl;
  xp.inv_scale = cw.inv_scale;
  xp.Fh = cw.Fh;
  xp.Fl = cw.Fl;
  xp.gn_rowpart = nullptr;
  xp.gn_cnt = 0;
  xp.gn_gamma = xp.gn_beta = nullptr;
  xp.gn_res = nullptr;
  xp.Uh = xp.Ul = nullptr;
  xp.u_bytes = 0;
  xp.a_amax = R.a_amax;
  xp.a_nparts = R.a_nparts;
  xp.w_inv = cw.inv_dev;
  {
    const size_t a_el = (size_t)N * p.Hin * p.Win * s.C;
    const size_t ab = a_el * (ash != nullptr ? 2 : 4), bb = (size_t)cw.npad * cw.kpad * 2;
    if (x3 && (ab >= ((size_t)1 << 31) || bb >= ((size_t)1 << 31)))
      throw Error(DMX_E_ARG, "gemm: operand too large for 32-bit buffer offsets (split the batch)");
    xp.a_bytes = (unsigned)ab;
    xp.b_bytes = (unsigned)bb;
  }
  // labels are the demangled kernel names rocprofv3 reports (profiles/ cross-check)
  const int sa = ash != nullptr ? 1 : 0;
  const int creal = (src_mode == SRC_NCHW && s.C0) ? s.C0 : cw.cin;
  const double flops = 2.0 * (double)M * cw.phases * cw.cout * (double)cw.taps * creal;
  const double bytes = 4.0 * ((double)M * cw.phases * cw.cout + (double)N * p.Hin * p.Win * s.C +
                              (double)cw.phases * cw.cout * cw.taps * cw.cin);
  char nm[96];
  auto name_x3 = [&](int e) {
    std::snprintf(nm, sizeof nm, "igemm_x3_kernel<%d, %d, %d, 64, 1, %d, %d>", bm, bn, e, sa, x1 ? 1 : 0);
  };
  auto name_f32 = [&](int e) {
    std::snprintf(nm, sizeof nm, "igemm_f32_kernel<%d, %d, %d, %d>", bm, bn, src_mode, e);
  };
  if (msbn) {  // low-resolution halo conv: 256-pixel tiles of whole samples (igemm_halo.h MS)
    const int e = splits > 1 ? (int)EPI_PARTIAL : (int)EPI_STATS;
    dim3 gm(cdiv(M, 256), cw.cout / msbn, splits);
    const bool cs = msbn == 64;
    if (cs) std::snprintf(nm, sizeof nm, "igemm_halo_cs_kernel<%d, %d, %d, %d>", e, sa, x1 ? 1 : 0, W);
    else std::snprintf(nm, sizeof nm, "igemm_halo_kernel<%d, %d, %d, %d, %d, 0>", msbn, e, sa, x1 ? 1 : 0, W);
    R.begin(nm, flops, bytes + (splits > 1 ? 4.0 * splits * M * cw.cout : 0.0));
    if (cs) launch_halo_cs(e, W, sa, x1 ? 1 : 0, xp, gm, R.st);
    else launch_halo_ms(e, msbn, W, sa, x1 ? 1 : 0, xp, gm, R.st);
    R.end();
    HIPCHK(hipGetLastError());
    if (splits == 1 || (defer != nullptr && defer->fused)) return rrows;
    SplitkParams q{partial, splits, M, cw.cout, cw.bias, res, out, rowpart, seg, epi, gelu_exact_flag(R)};
    const int rb = cdiv(M * (cw.cout / 4), 256);
    R.begin("splitk_reduce_kernel", 0.0, 4.0 * (double)(splits + 1) * M * cw.cout);
    splitk_reduce_kernel<<<rb, 256, 0, R.st>>>(q);
    R.end();
    HIPCHK(hipGetLastError());
    return rrows;
  }
  if (splits > 1 && !wino) {  // (split Winograd convs launch below with their own chunk units)
    dim3 grid(cdiv(M, bm), cdiv(cw.cout, bn), splits);
    if (x3) name_x3(EPI_PARTIAL);
    else name_f32(EPI_PARTIAL);
    R.begin(nm, flops, bytes + 4.0 * splits * M * cw.cout);
    if (x3) launch_x3_partial(bm, bn, sa, x1 ? 1 : 0, xp, grid, R.st);
    else launch_f32(src_mode, EPI_PARTIAL, bm, bn, p, grid, R.st);
    R.end();
    HIPCHK(hipGetLastError());
    if (defer != nullptr && defer->fused) return rrows;  // the caller's reduce_norm_kernel sums the slabs
    SplitkParams q{partial, splits, M, cw.cout, cw.bias, res, out, rowpart, seg, epi, gelu_exact_flag(R)};
    const int rb = cdiv(M * (cw.cout / 4), 256);
    R.begin("splitk_reduce_kernel", 0.0, 4.0 * (double)(splits + 1) * M * cw.cout);
    splitk_reduce_kernel<<<rb, 256, 0, R.st>>>(q);
    R.end();
    HIPCHK(hipGetLastError());
    return rrows;
  }
  if (hbn || wino) {  // halo-staged 3x3 conv, 256-pixel x hbn tiles (igemm_halo.h) / Winograd
    dim3 gh(M / 256, hbn ? cw.cout / hbn : 1, 1);
    const int gna = gn != nullptr ? (gn->res != nullptr ? 2 : 1) : 0;
    if (gna) {
      xp.gn_rowpart = gn->rowpart;
      xp.gn_cnt = gn->cnt;
      xp.gn_gamma = gn->gamma;
      xp.gn_beta = gn->beta;
      xp.gn_res = gn->res;
    }
    if (wino) {  // Winograd F(2x2, 3x3): 64 tiles (256 pixels) x 64 channels per block (igemm_wino.h)
      xp.Uh = cw.Uh;
      xp.Ul = cw.Ul;
      xp.u_bytes = (unsigned)((size_t)16 * cw.cout * s.C * 2);
      check_range(R, cw.Uh, xp.u_bytes, "U hi");
      check_range(R, cw.Ul, xp.u_bytes, "U lo");
      const int e = splits > 1 ? (int)EPI_PARTIAL : (int)EPI_STATS;
      if (x1) std::snprintf(nm, sizeof nm, "wino_kernel<%d, %d, %d, 1>", wg, gna, e);
      else std::snprintf(nm, sizeof nm, "wino_kernel<%d, %d, %d>", wg, gna, e);
      R.begin(nm, flops, bytes + (splits > 1 ? 4.0 * splits * M * cw.cout : 0.0));
      launch_wino(e, wg, gna, x1 ? 1 : 0, xp, dim3(wino_blocks(wg, N, H), cw.cout / 64, splits), R.st);
      R.end();
      HIPCHK(hipGetLastError());
      if (splits == 1 || (defer != nullptr && defer->fused)) return rrows;
      SplitkParams q{partial, splits, M, cw.cout, cw.bias, res, out, rowpart, seg, epi, gelu_exact_flag(R)};
      R.begin("splitk_reduce_kernel", 0.0, 4.0 * (double)(splits + 1) * M * cw.cout);
      splitk_reduce_kernel<<<cdiv(M * (cw.cout / 4), 256), 256, 0, R.st>>>(q);
      R.end();
      HIPCHK(hipGetLastError());
      return rrows;
    }
    std::snprintf(nm, sizeof nm, "igemm_halo_kernel<%d, %d, %d, %d, %d, %d>", hbn, (int)EPI_STATS, sa, x1 ? 1 : 0, W,
                  gna);
    R.begin(nm, flops, bytes);
    launch_halo(HALO_MODE, hbn, W, sa, x1 ? 1 : 0, gna, xp, gh, R.st);
    R.end();
    HIPCHK(hipGetLastError());
    return rrows;
  }
  if (pp) {  // 512-thread ping-pong kernel, 256 x bn tiles (igemm_pp.h)
    dim3 gpp(cdiv(M, 256), cdiv(cw.cout, bn), 1);
    std::snprintf(nm, sizeof nm, "igemm_pp_kernel<%d, %d, %d, %d>", bn, (int)EPI_STATS, sa, x1 ? 1 : 0);
    R.begin(nm, flops, bytes);
    launch_pp(bn, sa, x1 ? 1 : 0, xp, gpp, R.st);
    R.end();
    HIPCHK(hipGetLastError());
    return rrows;
  }
  dim3 grid(cdiv(M, bm), cdiv(cw.cout, bn), cw.phases);
  if (x3) name_x3(epi);
  else name_f32(epi == EPI_STATS ? epi : epi);
  R.begin(nm, flops, bytes);
  if (x3) {
    if (epi == EPI_STATS) launch_x3_stats(bm, bn, sa, x1 ? 1 : 0, xp, grid, R.st);
    else if (epi == EPI_BIAS || epi == EPI_BIAS_GELU || epi == EPI_BIAS_RES)
      launch_x3_epi(epi, bm, bn, sa, x1 ? 1 : 0, xp, grid, R.st);
    else throw Error(DMX_E_INTERNAL, "bad epilogue");
  } else {
    if (src_mode == SRC_NCHW && epi != EPI_STATS) throw Error(DMX_E_INTERNAL, "bad epilogue for NCHW source");
    launch_f32(src_mode, epi, bm, bn, p, grid, R.st);
  }
  R.end();
  HIPCHK(hipGetLastError());
  return rrows;
}

static void gn_finalize(Run& R, const float2* rowpart, float2* stats, int N, int rrows, int nseg, int G, int C,
                        int HWo) {
  if (R.plan) return;
  R.begin("gn_finalize_kernel", 0.0, 8.0 * (double)N * rrows * nseg);
  gn_finalize_kernel<<<N * G, 256, 0, R.st>>>(rowpart, stats, rrows, nseg, G, C, HWo, 1e-5f);
  R.end();
  HIPCHK(hipGetLastError());
}

// GroupNorm (+GELU | +residual GELU) (+emb) materialisation; stats inline (rowpart, G=1)
// or precomputed (stats).
static void norm(Run& R, NormParams np, int N) {
  if (R.plan) return;
  np.gexact = gelu_exact_flag(R);
  // ~2048+ blocks in total, 256..1024 float4 per block (chunks are rounded up to 256 in-kernel)
  const int per = np.HW * (np.C / 4);
  const int target = 1024;  // total blocks aimed at for small tensors (measured +0.3 % over 2048)
  const int chunks = std::max(1, std::min(cdiv(per, 256), std::max(cdiv(per, 1024), cdiv(target, N))));
  R.begin("norm_kernel", 0.0, 4.0 * (double)N * np.HW * np.C * (np.res ? 3 : 2));
  norm_kernel<<<dim3(chunks, N), 256, 0, R.st>>>(np);
  R.end();
  HIPCHK(hipGetLastError());
}

// Split-K slabs of a deferred GEMM -> GroupNorm(1, C) application (reduce_norm_kernel): one
// block per source sample; np describes the normalisation exactly as for norm().
static void reduce_norm(Run& R, const Deferred& d, NormParams np, int n_src_samples) {
  if (R.plan) return;
  np.gexact = gelu_exact_flag(R);
  const int kv = std::max(RN_MIN_KV, cdiv(np.HW * (np.C / 4), 1024));
  const int n_out = np.n_src > 0 ? 2 * n_src_samples : n_src_samples;
  const int kvt = kv <= 2 ? 2 : kv <= 4 ? 4 : RN_MAXV;
  R.begin("reduce_norm_kernel<" + std::to_string(kvt) + ">", 0.0,
          4.0 * (double)n_src_samples * np.HW * np.C * (d.splits + (np.res ? 1 : 0)) +
              4.0 * (double)n_out * np.HW * np.C);
  if (kv <= 2) reduce_norm_kernel<2><<<n_src_samples, 1024, 0, R.st>>>(d.partial, d.splits, d.bias, np);
  else if (kv <= 4) reduce_norm_kernel<4><<<n_src_samples, 1024, 0, R.st>>>(d.partial, d.splits, d.bias, np);
  else reduce_norm_kernel<RN_MAXV><<<n_src_samples, 1024, 0, R.st>>>(d.partial, d.splits, d.bias, np);
  R.end();
  HIPCHK(hipGetLastError());
}

template <int SRC>
static void prep(Run& R, const SrcDesc& s, float* out, int N, int H, int W, const char* name, _Float16* oh = nullptr,
                 _Float16* ol = nullptr) {
  if (R.plan) return;
  const size_t total = (size_t)N * H * W * (s.C / 4);
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 8192);
  R.begin(name, 0.0, 4.0 * (double)N * H * W * s.C * (SRC == SRC_MAXPOOL ? 5 : 2) * (oh ? 1.5 : 1.0));
  prep_kernel<SRC><<<blocks, 256, 0, R.st>>>(s, out, N, H, W, oh, ol);
  R.end();
  HIPCHK(hipGetLastError());
}

static SrcDesc plain_src(const float* p, int C) {
  SrcDesc s;
  std::memset(&s, 0, sizeof(s));
  s.src0 = p;
  s.C = C;
  s.G = 1;
  s.scale = 1.f;
  return s;
}

static NormParams norm_params(const float* raw, const float2* rowpart, int nseg, int rrows, const float* g,
                              const float* b, int C, int HW, float* out) {
  NormParams np;
  std::memset(&np, 0, sizeof(np));
  np.raw = raw;
  np.rowpart = rowpart;
  np.nseg = nseg;
  np.rrows = rrows;
  np.gamma = g;
  np.beta = b;
  np.C = C;
  np.G = 1;
  np.HW = HW;
  np.out = out;
  return np;
}

// ResBlock (models/unet_cond.py:10-30):
//   conv1 (+row stats) -> GN+GELU (materialised) -> conv2 (+row stats) -> GN [-> GELU(x + .)] [+ emb]
// `in` is a plain NHWC tensor (or the NCHW network input for `inc`); it doubles as the residual.
// n_out > N: the block is computed for N samples and its final GroupNorm (+ emb) writes
// n_out samples, output n reading sample n % N (the CFG-shared prefix of the trunk).
// in_h / in_l: `in` is available as f16 hi / lo planes (conv1 then reads those).
// planes_out: the output only feeds the next ResBlock's conv1 — write it as hi / lo planes
// (same bytes as fp32) when the split GEMM can use them; *wrote_planes reports the choice.
// defer_out (residual blocks whose conv2 wrote whole-sample partials): the final GroupNorm +
// residual + GELU is NOT launched; the raw conv2 output is returned and *defer_out describes the
// normalisation for the consumer (the next ResBlock's halo conv1, GNA = 2); defer_out->rowpart
// stays null when the block could not defer.  gn_in: `in` is such a deferred raw output (conv1
// applies it while staging; the block must not be residual).
static float* resblock(Run& R, const ResW& w, const SrcDesc& in, int mode, int N, int H, int W, bool residual,
                       const float* emb, int emb_stride, int emb_off, int n_out = 0,
                       const _Float16* in_h = nullptr, const _Float16* in_l = nullptr, bool planes_out = false,
                       bool* wrote_planes = nullptr, GnLoad* defer_out = nullptr, const GnLoad* gn_in = nullptr) {
  const int M = N * H * W, HW = H * W;
  if (n_out <= 0) n_out = N;
  const int seg = 32;
  float* r1 = R.ws.get<float>((size_t)M * w.mid);
  float2* rp1 = R.ws.get<float2>((size_t)M * (w.mid / seg));
  // conv2 on the Winograd kernel reads the fp32 mid activation (GroupNorm-on-load or materialised)
  const bool c2_wino = wino_any(R, w.mid, N, H, W, w.c2);
  const bool planes = R.m->prec >= 1 && split_a_enabled() && w.c2.Bh != nullptr && w.mid >= 64 && !c2_wino;
  float* a1 = R.ws.get<float>((size_t)M * w.mid);  // fp32 or, with planes, hi|lo f16 halves
  float* r2 = R.ws.get<float>((size_t)M * w.cout);
  float2* rp2 = R.ws.get<float2>((size_t)M * (w.cout / seg));
  float* out = R.ws.get<float>((size_t)n_out * HW * w.cout);
  Deferred d1, d2;  // split-K convs at low resolution: reduce + GroupNorm in one launch
  if (gn_in != nullptr && (residual || mode != SRC_PLAIN))
    throw Error(DMX_E_INTERNAL, "resblock: a GroupNorm-on-load input needs a plain, non-residual block");
  const int rr1 = gemm(R, in, mode, N, H, W, w.c1, EPI_STATS, r1, nullptr, rp1, seg, in_h, in_l, &d1, gn_in);
  NormParams n1 = norm_params(r1, rp1, w.mid / seg, rr1, w.g1.p, w.b1.p, w.mid, HW, a1);
  n1.act = 1;
  _Float16* a1h = reinterpret_cast<_Float16*>(a1);
  _Float16* a1l = a1h + (size_t)M * w.mid;
  if (planes) {
    n1.out = nullptr;
    n1.out_h = a1h;
    n1.out_l = a1l;
  }
  // The mid GroupNorm + GELU folded into conv2's halo staging (igemm_halo.h GNA) where conv2 runs
  // the halo conv and conv1 wrote whole-sample partials (no split-K slabs): no norm_kernel launch,
  // no hi / lo planes.  DMX_GN_FUSE=0 turns it off (the staged operand is the same either way).
  const bool fuse1 = gn_fuse_enabled() && !d1.fused && !R.m->debug &&
                     ((planes && halo_bn(R, w.mid, N, H, W, w.c2, EPI_STATS, true) > 0) ||
                      (c2_wino && wino_gna_pays(w.c2, 1, W)));
  int rr2;
  if (fuse1) {
    GnLoad g;
    g.rowpart = rp1;
    g.cnt = rr1 * (w.mid / seg);
    g.gamma = w.g1.p;
    g.beta = w.b1.p;
    rr2 = gemm(R, plain_src(r1, w.mid), SRC_PLAIN, N, H, W, w.c2, EPI_STATS, r2, nullptr, rp2, seg, nullptr, nullptr,
               &d2, &g);
  } else {
    if (d1.fused) reduce_norm(R, d1, n1, N);
    else norm(R, n1, N);
    rr2 = gemm(R, plain_src(a1, w.mid), SRC_PLAIN, N, H, W, w.c2, EPI_STATS, r2, nullptr, rp2, seg,
               planes ? a1h : nullptr, planes ? a1l : nullptr, &d2);
  }
  if (defer_out != nullptr) *defer_out = GnLoad{};
  if (defer_out != nullptr && residual && mode == SRC_PLAIN && !d2.fused && emb == nullptr && n_out == N &&
      !R.m->debug) {
    defer_out->rowpart = rp2;
    defer_out->cnt = rr2 * (w.cout / seg);
    defer_out->gamma = w.g2.p;
    defer_out->beta = w.b2.p;
    defer_out->res = in.src0;
    if (wrote_planes != nullptr) *wrote_planes = false;
    return r2;
  }
  NormParams n2 = norm_params(r2, rp2, w.cout / seg, rr2, w.g2.p, w.b2.p, w.cout, HW, out);
  if (residual) {
    if (mode != SRC_PLAIN) throw Error(DMX_E_INTERNAL, "residual ResBlock needs a plain input");
    n2.res = in.src0;
  }
  n2.emb = emb;
  n2.emb_stride = emb_stride;
  n2.emb_off = emb_off;
  n2.n_src = n_out > N ? N : 0;
  const bool pout = planes_out && R.m->prec >= 1 && split_a_enabled() && !R.m->debug && emb == nullptr &&
                    n_out == N && w.cout >= 64;
  if (wrote_planes != nullptr) *wrote_planes = pout;
  if (pout) {  // hi | lo halves of the output buffer, as a1
    n2.out = nullptr;
    n2.out_h = reinterpret_cast<_Float16*>(out);
    n2.out_l = n2.out_h + (size_t)n_out * HW * w.cout;
  }
  if (d2.fused) reduce_norm(R, d2, n2, N);
  else norm(R, n2, n_out);
  R.tap(R.layer + ".r1", r1, (size_t)M * w.mid);
  R.tap(R.layer, out, (size_t)n_out * HW * w.cout);
  return out;
}

static void layernorm(Run& R, const float* x, float* y, const Vec& w, const Vec& b, int M, int C) {
  if (R.plan) return;
  const int blocks = cdiv(M, 4);
  R.begin("layernorm_kernel<" + std::to_string(C / 64) + ">", 0.0, 8.0 * (double)M * C);
  switch (C) {
    case 64: layernorm_kernel<1><<<blocks, 256, 0, R.st>>>(x, y, w.p, b.p, M, 1e-5f); break;
    case 128: layernorm_kernel<2><<<blocks, 256, 0, R.st>>>(x, y, w.p, b.p, M, 1e-5f); break;
    case 256: layernorm_kernel<4><<<blocks, 256, 0, R.st>>>(x, y, w.p, b.p, M, 1e-5f); break;
    default: throw Error(DMX_E_INTERNAL, "layernorm: unsupported C");
  }
  R.end();
  HIPCHK(hipGetLastError());
}

// stats (training forward only): a softmax reference and 1 / sum per (sample, head, query) for the
// backward (train_engine.h attn_core_bwd; P = exp(s - ref) / sum holds for any reference)
static void attention_core(Run& R, const float* qkv, float* out, int N, int L, int C, float* stats = nullptr) {
  if (R.plan) return;
  const int D = C / 4;
  if (D != 16 && D != 32 && D != 64) throw Error(DMX_E_INTERNAL, "attention: unsupported head dim");
  // the split-precision cores: inference in modes 1 / 2, and the training forward (R.fwd_x3, with stats)
  const bool x3 = R.m->prec >= 1 || (R.fwd_x3 && stats != nullptr);
  if (stats != nullptr && R.m->prec == 2) throw Error(DMX_E_INTERNAL, "attention stats: not in fp16 mode");
  if (x3 && D == 16 && att16_lds_bytes(L, 0) <= 160 * 1024) {
    // head resident in LDS (sa5 / sa6): one block per (sample, head), no per-chunk staging
    const int x1 = R.m->prec == 2 ? 1 : 0, nw = L > 256 ? 16 : 8;
    R.begin("attention16_kernel<" + std::to_string(nw) + ", " + std::to_string(x1) + ">", 4.0 * N * (double)L * L * C,
            4.0 * (double)N * L * 4 * C);
    HIPCHK(launch_attention16(nw, x1, qkv, out, L, C, N, R.st, stats));
    R.end();
    HIPCHK(hipGetLastError());
    return;
  }
  if (x3) {
    dim3 grid(cdiv(L, 128), 4, N);
    const int x1 = R.m->prec == 2 ? 1 : 0, wpe = D == 16 ? 4 : 1;  // D = 16: >= 4 waves / SIMD (register cap)
    R.begin("attention_x3_kernel<" + std::to_string(D) + ", " + std::to_string(wpe) + ", " + std::to_string(x1) + ">",
            4.0 * N * (double)L * L * C, 4.0 * (double)N * L * 4 * C);
    launch_attention_x3(D, wpe, x1, qkv, out, L, C, grid, R.st, stats);
    R.end();
    HIPCHK(hipGetLastError());
    return;
  }
  const int qt = L >= 256 ? 2 : 1;
  dim3 grid(cdiv(L, 64 * qt), 4, N);
  R.begin("attention_kernel<" + std::to_string(D) + ", " + std::to_string(qt) + ">", 4.0 * N * (double)L * L * C,
          4.0 * (double)N * L * 4 * C);
  launch_attention_f32(D, qt, qkv, out, L, C, grid, R.st, stats);
  R.end();
  HIPCHK(hipGetLastError());
}

// Whether the C = 256 QKV runs tok_ln_qkv_w_kernel (8-wave blocks, 384 columns, the LayerNorm of a
// token tile twice instead of twelve times) instead of the 4-wave 64-column tok_ln_qkv_kernel: where
// its grid (two column halves per 64-token tile) still fills the chip — sa2 (8192 tokens: 35 vs 41 us
// eager), not sa3 (2048 tokens: 32 vs 14 us); everywhere was -0.2 % per CFG step (round 5 A/B).
// The choice follows the batch class (dec_n), not the raw token count, so a batch and its shards take
// the same kernel.  The two kernels also compute every output identically (the same
// tok_rows LayerNorm, the same k-step order), which test_large_batch_class_is_shard_exact guards.
static bool tok_qkv_wide(const Run& R, int N, int L) { return cdiv(dec_n(R, N) * L, 64) * 2 >= 256; }
static TokW tokw(const ConvW& c) { return TokW{c.Bh, c.Bl, c.bias, c.inv_scale, c.kpad, c.Fh, c.Fl}; }

// Fused token kernels (tokmlp.h) for the split-precision modes: TA -> attention core -> TB.
static float* attn_block_fused(Run& R, const AttnW& a, const float* x, int N, int H, int W) {
  const int C = a.c, M = N * H * W, L = H * W;
  float* qkv = R.ws.get<float>((size_t)M * 3 * C);
  float* ao = R.ws.get<float>((size_t)M * C);
  float* out = R.ws.get<float>((size_t)M * C);
  const int x1 = R.m->prec == 2 ? 1 : 0;
  if (!R.plan) {
    TokParams tp{};
    tp.x = x;
    tp.M = M;
    tp.l1w = a.l1w.p;
    tp.l1b = a.l1b.p;
    tp.l2w = a.l2w.p;
    tp.l2b = a.l2b.p;
    const std::string cs = std::to_string(C);
    tp.out = qkv;
    tp.w0 = tokw(a.qkv);
    if (C == 64 || C == 128) {
      // in_proj slice resident in LDS, up to 4 token tiles per block; C = 64: all 3C = 192 columns per block
      const int nbl = C == 64 ? 192 : 64, gy = 3 * C / nbl, tiles = cdiv(M, 64);
      const int tpb = cdiv(tiles, 4) * gy >= 512 ? 4 : cdiv(tiles, 2) * gy >= 512 ? 2 : 1;
      const dim3 gl(cdiv(tiles, tpb), gy);
      R.begin("tok_ln_qkv_lds_kernel<" + cs + ", " + std::to_string(nbl) + ", " + std::to_string(tpb) + ", " +
                  std::to_string(x1) + ">",
              2.0 * M * C * 3.0 * C, 16.0 * (double)M * C);
      launch_tok_qkv_lds(C, tpb, x1, tp, gl, R.st);
    } else if (tok_qkv_wide(R, N, L)) {
      // C = 256: 8-wave blocks of 64 tokens x 384 columns (one round of blocks, LayerNorm twice per tile)
      const dim3 grid(cdiv(M, 64), 2);
      R.begin("tok_ln_qkv_w_kernel<" + cs + ", 384, 8, 4, " + std::to_string(x1) + ">", 2.0 * M * C * 3.0 * C,
              16.0 * (double)M * C);
      launch_tok_qkv_w(C, x1, tp, grid, R.st);
    } else {
      const int nb = 64;  // C = 256: 64 columns per block doubles the grid (M <= 8192 here)
      const dim3 grid(cdiv(M, 64), 3 * C / nb);
      R.begin("tok_ln_qkv_kernel<" + cs + ", " + std::to_string(nb) + ", " + std::to_string(x1) + ">",
              2.0 * M * C * 3.0 * C, 16.0 * (double)M * C);
      launch_tok_qkv(C, nb, x1, tp, grid, R.st);
    }
    R.end();
    HIPCHK(hipGetLastError());
  }
  attention_core(R, qkv, ao, N, L, C);
  if (!R.plan) {
    TokParams tp{};
    tp.x = x;
    tp.ao = ao;
    tp.out = out;
    tp.M = M;
    tp.l1w = a.l1w.p;
    tp.l1b = a.l1b.p;
    tp.l2w = a.l2w.p;
    tp.l2b = a.l2b.p;
    tp.w0 = tokw(a.o);
    tp.w1 = tokw(a.f1);
    tp.w2 = tokw(a.f2);
    // 32-token tiles when 64-token tiles would leave the chip under-filled (or C = 256)
    const int tm = C == 64 ? 64 : (C == 256 || cdiv(M, 64) < 512) ? 32 : 64;
    const bool lds64 = C == 64;  // weights in LDS, 128-token tiles, 8 waves, several tiles / block
    const int tiles128 = cdiv(M, 128), tpb = lds64 ? (tiles128 >= 1024 ? 4 : tiles128 >= 512 ? 2 : 1) : 1;
    const int nw = C == 256 ? 8 : lds64 ? 8 : 4;
    const int tmk = lds64 ? 128 : tm;
    const int blocks = lds64 ? cdiv(tiles128, tpb) : cdiv(M, tm);
    R.begin("tok_attn_out_kernel<" + std::to_string(C) + ", " + std::to_string(tmk) + ", " + std::to_string(x1) +
                ", " + std::to_string(nw) + ", " + std::to_string(lds64 ? 1 : 0) + ", " + std::to_string(tpb) + ">",
            6.0 * M * (double)C * C, 12.0 * (double)M * C);
    launch_tok_out(C, tm, x1, nw, lds64 ? 1 : 0, tpb, tp, blocks, R.st);
    R.end();
    HIPCHK(hipGetLastError());
  }
  R.tap(R.layer + ".qkv", qkv, (size_t)M * 3 * C);
  R.tap(R.layer + ".ao", ao, (size_t)M * C);
  R.tap(R.layer, out, (size_t)M * C);
  return out;
}

// AttenionBlock (models/unet_cond.py:32-52) on NHWC == (N, L, C) tokens.
static float* attn_block(Run& R, const AttnW& a, const float* x, int N, int H, int W) {
  const int C = a.c, M = N * H * W, L = H * W;
  if (R.m->prec >= 1 && (C == 64 || C == 128 || C == 256) && a.qkv.kpad == C &&
      a.o.kpad == C && a.f1.kpad == C && a.f2.kpad == C)
    return attn_block_fused(R, a, x, N, H, W);
  float* xl = R.ws.get<float>((size_t)M * C);
  float* qkv = R.ws.get<float>((size_t)M * 3 * C);
  float* ao = R.ws.get<float>((size_t)M * C);
  float* av = R.ws.get<float>((size_t)M * C);
  float* al = R.ws.get<float>((size_t)M * C);
  float* f = R.ws.get<float>((size_t)M * C);
  float* out = R.ws.get<float>((size_t)M * C);
  layernorm(R, x, xl, a.l1w, a.l1b, M, C);
  gemm(R, plain_src(xl, C), SRC_PLAIN, N, H, W, a.qkv, EPI_BIAS, qkv, nullptr, nullptr, 1);
  attention_core(R, qkv, ao, N, L, C);
  gemm(R, plain_src(ao, C), SRC_PLAIN, N, H, W, a.o, EPI_BIAS_RES, av, xl, nullptr, 1);
  layernorm(R, av, al, a.l2w, a.l2b, M, C);
  gemm(R, plain_src(al, C), SRC_PLAIN, N, H, W, a.f1, EPI_BIAS_GELU, f, nullptr, nullptr, 1);
  gemm(R, plain_src(f, C), SRC_PLAIN, N, H, W, a.f2, EPI_BIAS_RES, out, av, nullptr, 1);
  R.tap(R.layer + ".xl", xl, (size_t)M * C);
  R.tap(R.layer + ".qkv", qkv, (size_t)M * 3 * C);
  R.tap(R.layer + ".ao", ao, (size_t)M * C);
  R.tap(R.layer + ".av", av, (size_t)M * C);
  R.tap(R.layer, out, (size_t)M * C);
  return out;
}

struct FwdIn {
  const float* x;        // NCHW (n_x samples)
  int n_x;               // samples in x (N or N/2 under CFG batching)
  const int64_t* t; int t_stride;
  const int64_t* y; int y_null_first; int64_t y_null;
  const float* vals; const float* mask; int cond_rows;
  int64_t* t_next = nullptr;  // multi-step graphs: where the embedding kernel stores t - 1
  bool cond_cached = false;   // multi-step graphs, steps after the first: the cond-MLP rows are
                              // already in the workspace (t-independent, same address every step)
};

// UnetCond trunk (models/unet_cond_geom.py:52-76): returns the (N,H,W,64) feature
static float* unet_trunk(Run& R, const FwdIn& in, int N, int H, int W) {
  dmx_model* m = R.m;
  // embedding
  float* emb = R.ws.get<float>((size_t)N * m->hsum);
  const bool has_cond = m->kind != DMX_UNET && in.vals != nullptr;
  const int cond_rows = in.cond_rows > 0 ? in.cond_rows : N;
  float* cnd = has_cond ? R.ws.get<float>((size_t)cond_rows * 256) : nullptr;
  if (!R.plan) {
    EmbedParams e;
    std::memset(&e, 0, sizeof(e));
    e.t = in.t;
    e.t_stride = in.t_stride;
    e.t_next = in.t_stride == 0 ? in.t_next : nullptr;
    e.t_mod = in.n_x < N ? in.n_x : 0;
    e.tmax = m->ctx->tmax;
    e.y = m->kind == DMX_UNET ? nullptr : in.y;
    e.y_null_first = in.y_null_first;
    e.y_null = in.y_null;
    e.n_half = in.y_null_first ? N / 2 : N;
    e.vals = m->kind == DMX_UNET ? nullptr : in.vals;
    e.mask = in.mask;
    e.cond_rows = in.cond_rows > 0 ? in.cond_rows : N;
    e.pos_table = m->ctx->pos_table;
    e.class_emb = m->class_emb;
    e.ncls = m->cfg.ncls;
    e.w0 = m->w0;
    e.b0 = m->b0;
    e.w2t = m->w2t;
    e.b2 = m->b2;
    e.wht = m->wht;
    e.bh = m->bh;
    e.hsum = m->hsum;
    e.out = emb;
    R.layer = "embed";
    if (has_cond) {  // cond_mlp once per distinct condition row (the CFG halves share it)
      if (!in.cond_cached) {
        R.begin("cond_emb_kernel", 2.0 * cond_rows * (24.0 * 256 + 256.0 * 256), 4.0 * (256.0 * 256 + 24.0 * 256));
        cond_emb_kernel<<<cond_rows, 256, 0, R.st>>>(e, cnd);
        R.end();
        HIPCHK(hipGetLastError());
      }
      e.cnd = cnd;
    }
    R.begin("embed_kernel", 2.0 * N * (24.0 * 256 + 256.0 * 256 + 256.0 * m->hsum), 4.0 * (256.0 * 256 + 256.0 * m->hsum));
    embed_kernel<<<dim3(N, cdiv(m->hsum, 256)), 256, 0, R.st>>>(e);
    R.end();
    R.tap("emb", emb, (size_t)N * m->hsum);
    HIPCHK(hipGetLastError());
  }
  // CFG batching (samples [0, S) and [S, 2S) share x and t, differ in y / cond): nothing
  // before the first embedding add depends on y, so inc and down1's two ResBlocks run once
  // for S samples and down1's final GroupNorm + emb add fans out to all N
  // (models/unet_cond.py:63-68, Down.forward: maxpool_conv(x) + emb).  Exact: the shared
  // values are the ones the reference computes twice.
  const int S = in.n_x < N ? in.n_x : N;
  SrcDesc xs = plain_src(in.x, m->inc.cin);
  xs.C0 = m->in_ch;
  R.layer = "inc";
  float* x1 = resblock(R, m->inc, xs, SRC_NCHW, S, H, W, false, nullptr, 0, 0);
  // down path: skips x1 (H), a1 (H/2), a2 (H/4)
  const float* skips[3];
  int sh[3], sw[3], sc[3];
  const float* cur = x1;
  int ch = H, cw = W, cc = 64;
  for (int i = 0; i < 3; ++i) {
    skips[i] = cur;
    sh[i] = ch;
    sw[i] = cw;
    sc[i] = cc;
    SrcDesc mp = plain_src(cur, cc);
    mp.Hs = ch;
    mp.Ws = cw;
    const int nh = ch / 2, nw = cw / 2;
    const int nb = i == 0 ? S : N;  // samples computed in this stage before the emb add
    R.layer = "down" + std::to_string(i + 1) + ".0";
    const size_t pool_el = (size_t)nb * nh * nw * cc;
    float* pooled = R.ws.get<float>(pool_el);
    const bool pool_planes = R.m->prec >= 1 && m->down[i].r0.c1.Bh != nullptr && !R.m->debug && cat_planes_enabled() &&
                             !((halo_bn(R, cc, nb, nh, nw, m->down[i].r0.c1, EPI_STATS, true) > 0 ||
                                                          halo_ms_bn_any(R, cc, nb, nh, nw, m->down[i].r0.c1))) &&
                             !wino_any(R, cc, nb, nh, nw, m->down[i].r0.c1);
    _Float16* pool_h = pool_planes ? R.ws.get<_Float16>(2 * pool_el) : nullptr;
    _Float16* pool_l = pool_planes ? pool_h + pool_el : nullptr;
    prep<SRC_MAXPOOL>(R, mp, pooled, nb, nh, nw, "prep_kernel<2>", pool_h, pool_l);
    bool hp = false;
    float* h0 = resblock(R, m->down[i].r0, plain_src(pooled, cc), SRC_PLAIN, nb, nh, nw, true, nullptr, 0, 0, 0,
                         pool_h, pool_l, m->down[i].r1.c1.Bh != nullptr && !wino_any(R, cc, nb, nh, nw, m->down[i].r1.c1),
                         &hp);
    R.layer = "down" + std::to_string(i + 1) + ".1";
    const _Float16* h0h = hp ? reinterpret_cast<const _Float16*>(h0) : nullptr;
    float* h1 = resblock(R, m->down[i].r1, plain_src(h0, cc), SRC_PLAIN, nb, nh, nw, false, emb, m->hsum,
                         m->down[i].emb_off, N, h0h, hp ? h0h + (size_t)nb * nh * nw * cc : nullptr);
    cc = m->down[i].cout;
    ch = nh;
    cw = nw;
    R.layer = "sa" + std::to_string(i + 1);
    cur = attn_block(R, m->sa[i], h1, N, ch, cw);
  }
  // bottleneck
  const _Float16 *cur_h = nullptr, *cur_l = nullptr;  // planes of `cur` (between bottleneck blocks)
  for (int i = 0; i < m->nbot; ++i) {
    R.layer = "bot" + std::to_string(i + 1);
    bool hp = false;
    const bool nxt = i + 1 < m->nbot && m->bot[i + 1].c1.Bh != nullptr &&  // the last one feeds the upsample
                     !wino_any(R, m->bot[i].cout, N, ch, cw, m->bot[i + 1].c1);
    cur = resblock(R, m->bot[i], plain_src(cur, cc), SRC_PLAIN, N, ch, cw, false, nullptr, 0, 0, 0, cur_h, cur_l, nxt,
                   &hp);
    cc = m->bot[i].cout;
    cur_h = hp ? reinterpret_cast<const _Float16*>(cur) : nullptr;
    cur_l = hp ? cur_h + (size_t)N * ch * cw * cc : nullptr;
  }
  // up path
  for (int i = 0; i < 3; ++i) {
    const int si = 2 - i;  // skip x3, x2, x1
    SrcDesc u = plain_src(skips[si], sc[si] + cc);
    u.C0 = sc[si];
    u.n_mod = si == 0 && S < N ? S : 0;  // x1 was computed once for both CFG halves
    u.src1 = cur;
    u.Hs = ch;
    u.Ws = cw;
    const int dy = sh[si] - 2 * ch, dx = sw[si] - 2 * cw;
    u.padT = dy > 0 ? dy / 2 : 0;
    u.padL = dx > 0 ? dx / 2 : 0;
    REQUIRE(u.C == m->up[i].r0.cin, "up: channel mismatch");
    R.layer = "up" + std::to_string(i + 1) + ".0";
    const size_t cat_el = (size_t)N * sh[si] * sw[si] * u.C;
    float* cat = R.ws.get<float>(cat_el);
    // the concat feeds conv1 (split GEMM: also as f16 planes) and the residual (fp32)
    const bool cat_planes = R.m->prec >= 1 && m->up[i].r0.c1.Bh != nullptr && !R.m->debug && cat_planes_enabled() &&
                            !((halo_bn(R, u.C, N, sh[si], sw[si], m->up[i].r0.c1, EPI_STATS, true) > 0 ||
                                                         halo_ms_bn_any(R, u.C, N, sh[si], sw[si], m->up[i].r0.c1))) &&
                            !wino_any(R, u.C, N, sh[si], sw[si], m->up[i].r0.c1);
    _Float16* cat_h = cat_planes ? R.ws.get<_Float16>(2 * cat_el) : nullptr;
    _Float16* cat_l = cat_planes ? cat_h + cat_el : nullptr;
    prep<SRC_UPCAT>(R, u, cat, N, sh[si], sw[si], "prep_kernel<3>", cat_h, cat_l);
    bool hp = false;
    // r0's final GroupNorm + residual + GELU folded into r1's halo conv1 where that conv runs the
    // halo kernel (igemm_halo.h GNA = 2): one norm_kernel launch and the h0 round trip fewer
    GnLoad dly;
    const bool r1_wino = wino_any(R, u.C, N, sh[si], sw[si], m->up[i].r1.c1);
    const bool try_defer = gn_fuse_enabled() && !R.m->debug && R.m->prec >= 1 &&
                           (r1_wino ? wino_gna_pays(m->up[i].r1.c1, 2, sw[si])
                                    : halo_bn(R, u.C, N, sh[si], sw[si], m->up[i].r1.c1, EPI_STATS, true) > 0);
    float* h0 = resblock(R, m->up[i].r0, plain_src(cat, u.C), SRC_PLAIN, N, sh[si], sw[si], true, nullptr, 0, 0, 0,
                         cat_h, cat_l, m->up[i].r1.c1.Bh != nullptr && !r1_wino, &hp, try_defer ? &dly : nullptr);
    R.layer = "up" + std::to_string(i + 1) + ".1";
    const _Float16* h0h = hp ? reinterpret_cast<const _Float16*>(h0) : nullptr;
    float* h1 = dly.rowpart != nullptr
                    ? resblock(R, m->up[i].r1, plain_src(h0, u.C), SRC_PLAIN, N, sh[si], sw[si], false, emb, m->hsum,
                               m->up[i].emb_off, 0, nullptr, nullptr, false, nullptr, nullptr, &dly)
                    : resblock(R, m->up[i].r1, plain_src(h0, u.C), SRC_PLAIN, N, sh[si], sw[si], false, emb, m->hsum,
                               m->up[i].emb_off, 0, h0h, hp ? h0h + (size_t)N * sh[si] * sw[si] * u.C : nullptr);
    ch = sh[si];
    cw = sw[si];
    cc = m->up[i].cout;
    R.layer = "sa" + std::to_string(4 + i);
    cur = attn_block(R, m->sa[3 + i], h1, N, ch, cw);
  }
  return const_cast<float*>(cur);
}

static void check_shapes(dmx_model* m, int n, int h, int w) {
  if (!m->finalized) throw Error(DMX_E_STATE, "model weights not finalized");
  if (m->kind == DMX_VAE) throw Error(DMX_E_ARG, "not a U-Net model");
  REQUIRE(n >= 1, "batch must be >= 1");
  REQUIRE(h >= 8 && w >= 8, "latent must be at least 8x8");
  REQUIRE(h == w, "AttenionBlock assumes square maps (models/unet_cond.py:46-47)");
  REQUIRE(m->ctx->pos_table != nullptr, "time table not set (dmx_set_time_table)");
}

static void drop_graph(dmx_model* m) {
  if (m->has_graph) {
    (void)hipGraphExecDestroy(m->gexec);
    (void)hipGraphDestroy(m->graph);
    if (m->gexec_k) (void)hipGraphExecDestroy(m->gexec_k);
    if (m->graph_k) (void)hipGraphDestroy(m->graph_k);
    m->gexec_k = nullptr;
    m->graph_k = nullptr;
    m->has_graph = false;
  }
}

// Re-derive the f16 planes of the split GEMMs after dmx_model_refresh (weights changed in
// place), before the next split-precision launch; captured graphs hold the old scales.
static void ensure_planes(dmx_model* m, hipStream_t st) {
  if (!m->planes_stale || m->prec < 1) return;
  drop_graph(m);
  for_each_conv(m, [&](ConvW& c) {
    if (c.Bh != nullptr) split_planes(c, st, m->amax);
  });
  m->planes_stale = false;
}

// Diagnostic (DMX_POISON=1): fill every workspace with 0xFF bytes (fp32 NaN) before the real
// pass, so a kernel reading an element no earlier kernel of the same run wrote turns the
// outputs non-finite instead of silently reusing stale data.
static bool poison_ws() {
  static const bool v = [] {
    const char* e = std::getenv("DMX_POISON");
    return e != nullptr && std::atoi(e) != 0;
  }();
  return v;
}
static void poison(void* mem, size_t bytes, hipStream_t st) {
  if (poison_ws() && mem != nullptr && bytes > 0) HIPCHK(hipMemsetAsync(mem, 0xFF, bytes, st));
}

static void ensure_ws(dmx_model* m) {
  if (m->ws.off > m->ws_cap) {
    if (m->ws_mem) HIPCHK(hipFree(m->ws_mem));
    m->ws_mem = nullptr;
    m->ws_cap = 0;
    drop_graph(m);
    HIPCHK(hipMalloc(&m->ws_mem, m->ws.off));
    m->ws_cap = m->ws.off;
  }
}

template <typename F>
static void run_planned(dmx_model* m, hipStream_t st, F&& body) {
  m->ws.base = nullptr;
  m->ws.off = 0;
  m->ws.plan = true;
  {
    Run R{m, st, true, m->ws};
    body(R);
  }
  ensure_ws(m);
  const size_t planned = m->ws.off;
  poison(m->ws_mem, m->ws.off, st);
  m->ws.base = static_cast<char*>(m->ws_mem);
  m->ws.off = 0;
  m->ws.plan = false;
  Cksum& ck = cksum_state();
  if (cksum_enabled()) {
    if (ck.dev == nullptr) HIPCHK(hipMalloc(&ck.dev, 1024 * sizeof(unsigned long long)));
    HIPCHK(hipMemsetAsync(ck.dev, 0, 1024 * sizeof(unsigned long long), st));
    HIPCHK(hipMemsetAsync(m->ws_mem, 0xFF, planned, st));
    ck.names.clear();
  }
  Run R{m, st, false, m->ws};
  R.cksum = cksum_enabled();
  body(R);
  if (m->ws.off != planned) throw Error(DMX_E_INTERNAL, "workspace plan / run mismatch");
  if (cksum_enabled()) {
    R.ck();
    std::vector<unsigned long long> h(ck.names.size());
    HIPCHK(hipMemcpyAsync(h.data(), ck.dev, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (ck.names == ck.prev_names) {
      for (size_t k = 0; k < h.size(); ++k)
        if (h[k] != ck.prev[k]) {
          std::fprintf(stderr, "[dmx cksum] run %d: first difference after kernel %zu (%s)\n", ck.runs, k,
                       ck.names[k].c_str());
          break;
        }
    }
    ck.prev = h;
    ck.prev_names = ck.names;
    ++ck.runs;
  }
}

// t_next (multi-step sample-loop graphs): the step's t - 1 is stored there by the embedding kernel.
static void step_body(Run& R, const dmx_step_args& a, int64_t* t_next = nullptr, bool cond_cached = false) {
  dmx_model* m = R.m;
  const bool cfg = m->kind != DMX_UNET && a.guidance > 0.f && a.y != nullptr;
  const int N = cfg ? 2 * a.n : a.n;
  FwdIn in{a.x_in, a.n, a.t, a.t_stride, a.y, cfg ? 1 : 0, a.null_label, a.vals, a.mask, a.n};
  in.t_next = t_next;
  in.cond_cached = cond_cached;
  float* feat = unet_trunk(R, in, N, a.h, a.w);
  if (R.plan) return;
  StepTailParams p;
  std::memset(&p, 0, sizeof(p));
  p.feat = feat;
  p.w = m->out_w;
  p.b = m->out_b;
  p.Co = m->in_ch;
  p.B = a.n;
  p.HW = a.h * a.w;
  p.cfg = cfg ? 1 : 0;
  p.guidance = a.guidance;
  p.x = a.x_in;
  p.x_out = a.x_out;
  p.t = a.t;
  p.t_stride = a.t_stride;
  p.tmax = a.T;
  p.c1 = a.c1;
  p.c2 = a.c2;
  p.sd = a.sd;
  p.noise = a.noise;
  p.seed = a.seed;
  p.sample_offset = a.sample_offset;
  p.range_flag = m->range_flag;
  R.layer = "out+cfg+ddpm";
  if (p.Co == 4 && p.feat != nullptr) {
    dim3 grid(cdiv(p.HW, 16), a.n);
    R.begin("step_tail4_kernel", 2.0 * N * p.HW * 64.0 * p.Co, 4.0 * ((double)N * p.HW * 64 + 3.0 * a.n * p.HW * p.Co));
    step_tail4_kernel<<<grid, 256, 0, R.st>>>(p);
  } else {
    dim3 grid(cdiv(p.HW, 256), a.n);
    R.begin("step_tail_kernel", 2.0 * N * p.HW * 64.0 * p.Co, 4.0 * ((double)N * p.HW * 64 + 3.0 * a.n * p.HW * p.Co));
    step_tail_kernel<<<grid, 256, 0, R.st>>>(p);
  }
  R.end();
  HIPCHK(hipGetLastError());
}

static void validate_step(dmx_model* m, const dmx_step_args* a) {
  REQUIRE(a != nullptr, "null step args");
  check_shapes(m, a->n, a->h, a->w);
  REQUIRE(a->x_in && a->x_out && a->t && a->c1 && a->c2 && a->sd, "null tensor in step args");
  REQUIRE(a->T >= 1, "T must be >= 1");
  REQUIRE(m->in_ch <= 4, "in_ch must be <= 4");
  if (m->kind != DMX_UNET && a->guidance > 0.f) REQUIRE(a->y != nullptr, "CFG needs y");
  if (m->kind == DMX_UNET_COND_GEOM || m->kind == DMX_UNET_COND)
    REQUIRE((a->vals == nullptr) == (a->mask == nullptr), "vals and mask must be given together");
}

// VAE decoder (models/vae.py:35-49,64-69) on one chunk of n latents:
// [conv3x3 | ConvT-phase GEMM] (+row stats) -> GN(8) finalize -> GN+GELU materialised, x6, then
// conv3x3 64->3 + sigmoid + uint8 in vae_tail_kernel.
static void vae_body(Run& R, const float* z, float* img, uint8_t* u8, int n, int h, int w) {
  dmx_model* m = R.m;
  const int G = 8;
  R.tile_n = 1;  // per-sample tiling decisions: decoded bytes independent of the batch / chunk
  SrcDesc s = plain_src(z, 4);
  s.C0 = 4;
  s.scale = m->cfg.scale;
  int mode = SRC_NCHW;
  int H = h, W = w;
  const float* act = nullptr;
  for (int stage = 0; stage < 6; ++stage) {
    const bool convt = stage & 1;
    const ConvW& cw = convt ? m->vconvt[stage / 2] : m->vconv[stage / 2];
    const int Ho = convt ? 2 * H : H, Wo = convt ? 2 * W : W;
    const int Mo = n * Ho * Wo;
    const int seg = std::min(32, cw.cout / G);
    R.layer = "dec" + std::to_string(stage);
    float* r = R.ws.get<float>((size_t)Mo * cw.cout);
    float2* rp = R.ws.get<float2>((size_t)Mo * (cw.cout / seg));
    float2* st = R.ws.get<float2>((size_t)n * G);
    float* a = R.ws.get<float>((size_t)Mo * cw.cout);
    const int rr = gemm(R, s, mode, n, H, W, cw, EPI_STATS, r, nullptr, rp, seg);
    gn_finalize(R, rp, st, n, rr, cw.cout / seg, G, cw.cout, Ho * Wo);
    NormParams np = norm_params(r, nullptr, 0, 0, m->vg[stage].p, m->vb[stage].p, cw.cout, Ho * Wo, a);
    np.stats = st;
    np.G = G;
    np.act = 1;
    norm(R, np, n);
    act = a;
    s = plain_src(a, cw.cout);
    mode = SRC_PLAIN;
    H = Ho;
    W = Wo;
  }
  R.tile_n = 0;
  if (R.plan) return;
  dim3 grid(cdiv(H * W, 256), n);
  R.begin("vae_tail_kernel", 2.0 * n * H * W * 3 * 576, 4.0 * (double)n * H * W * (64 + 3) + (double)n * H * W * 3);
  vae_tail_kernel<<<grid, 256, 0, R.st>>>(act, m->vconv[3].B, m->vconv[3].bias, n, H, W, img, u8, m->range_flag);
  R.end();
  HIPCHK(hipGetLastError());
}

// VAE encoder (models/vae.py:17-30, 51-62) on n images (n,3,h,w), h, w multiples of 8:
// [conv3x3 | conv4x4-s2 GEMM] (+row stats) -> GN(8) finalize -> GN+GELU materialised, x6, then
// the 1x1 mu / logvar heads + reparameterisation + per-sample KL in vae_enc_tail_kernel.
static void vae_enc_body(Run& R, const float* x, const float* eps, float* z, float* kl, int n, int h, int w) {
  dmx_model* m = R.m;
  const int G = 8;
  SrcDesc s = plain_src(x, 4);  // NCHW image, 3 real channels padded to 4
  s.C0 = 3;
  int mode = SRC_NCHW;
  int H = h, W = w;
  const float* act = nullptr;
  for (int stage = 0; stage < 6; ++stage) {
    const bool strided = stage & 1;
    const ConvW& cw = m->venc[stage];
    const int Ho = strided ? H / 2 : H, Wo = strided ? W / 2 : W;
    const int Mo = n * Ho * Wo;
    const int seg = std::min(32, cw.cout / G);
    R.layer = "enc" + std::to_string(stage);
    float* r = R.ws.get<float>((size_t)Mo * cw.cout);
    float2* rp = R.ws.get<float2>((size_t)Mo * (cw.cout / seg));
    float2* st = R.ws.get<float2>((size_t)n * G);
    float* a = R.ws.get<float>((size_t)Mo * cw.cout);
    const int rr = gemm(R, s, mode, n, Ho, Wo, cw, EPI_STATS, r, nullptr, rp, seg);  // rows = output pixels
    gn_finalize(R, rp, st, n, rr, cw.cout / seg, G, cw.cout, Ho * Wo);
    NormParams np = norm_params(r, nullptr, 0, 0, m->veg[stage].p, m->veb[stage].p, cw.cout, Ho * Wo, a);
    np.stats = st;
    np.G = G;
    np.act = 1;
    norm(R, np, n);
    R.tap(R.layer, a, (size_t)Mo * cw.cout);
    act = a;
    s = plain_src(a, cw.cout);
    mode = SRC_PLAIN;
    H = Ho;
    W = Wo;
  }
  const int nb = cdiv(H * W, 32);
  float* klp = R.ws.get<float>((size_t)n * nb);
  if (R.plan) return;
  R.begin("vae_enc_tail_kernel", 2.0 * n * H * W * 8 * 256, 4.0 * (double)n * H * W * (256 + 4 + 4));
  vae_enc_tail_kernel<<<dim3(nb, n), 256, 0, R.st>>>(act, m->wmu, m->bmu, m->wlv, m->blv, eps, z, klp, H * W,
                                                      m->cfg.scale, m->range_flag);
  vae_enc_kl_kernel<<<cdiv(n, 64), 64, 0, R.st>>>(klp, nb, n, 1.0f / ((float)h * (float)w), kl);
  R.end();
  HIPCHK(hipGetLastError());
}

}  // namespace dmx

#include "train_engine.h"

// ===========================================================================
// C ABI
// ===========================================================================
using namespace dmx;

template <typename F>
static int guarded(F&& f) {
  try {
    f();
    return DMX_OK;
  } catch (const Error& e) {
    g_err = e.what();
    return e.code;
  } catch (const std::exception& e) {
    g_err = e.what();
    return DMX_E_INTERNAL;
  } catch (...) {
    g_err = "unknown error";
    return DMX_E_INTERNAL;
  }
}

static ModelCfg to_cfg(const dmx_model_config& c) {
  ModelCfg m;
  REQUIRE(c.kind >= DMX_UNET_COND_GEOM && c.kind <= DMX_VAE, "unknown model kind");
  REQUIRE(c.in_ch >= 1 && c.in_ch <= 4, "in_ch must be in [1,4]");
  REQUIRE(c.num_classes >= 0 && c.num_classes < (1 << 20), "bad num_classes");
  REQUIRE(c.geom_dim >= 1 && c.geom_dim <= 4096 && c.geom_hidden >= 1 && c.geom_hidden <= 4096,
          "geom_dim / geom_hidden must be in [1, 4096]");
  REQUIRE(std::isfinite(c.scale_factor) && c.scale_factor != 0.f, "scale_factor must be finite and non-zero");
  m.kind = c.kind;
  m.in_ch = c.in_ch;
  m.deep = !c.remove_deep_conv;
  m.ncls = c.num_classes + 1;
  m.gdim = c.geom_dim;
  m.ghid = c.geom_hidden;
  m.scale = c.scale_factor;
  return m;
}

static dmx_model_config default_cfg(int kind, int in_ch, int remove_deep_conv) {
  dmx_model_config c;
  c.kind = kind;
  c.in_ch = in_ch;
  c.remove_deep_conv = remove_deep_conv;
  c.num_classes = 3;
  c.geom_dim = 12;
  c.geom_hidden = 256;
  c.scale_factor = 0.18215f;
  return c;
}

extern "C" {

int dmx_abi_version(void) { return 1; }
const char* dmx_last_error(void) { return g_err.c_str(); }

int dmx_create(int device, dmx_ctx** out) {
  return guarded([&] {
    REQUIRE(out != nullptr, "null out");
    HIPCHK(hipSetDevice(device));
    auto* c = new dmx_ctx();
    c->device = device;
    *out = c;
  });
}

int dmx_destroy(dmx_ctx* ctx) {
  return guarded([&] {
    if (!ctx) return;
    if (ctx->pos_table) (void)hipFree(ctx->pos_table);
    delete ctx;
  });
}

int dmx_set_time_table(dmx_ctx* ctx, const float* host_table, int tmax) {
  return guarded([&] {
    REQUIRE(ctx && host_table && tmax >= 1, "bad time table");
    if (ctx->pos_table) HIPCHK(hipFree(ctx->pos_table));
    ctx->pos_table = nullptr;
    HIPCHK(hipMalloc(&ctx->pos_table, (size_t)tmax * 256 * sizeof(float)));
    HIPCHK(hipMemcpy(ctx->pos_table, host_table, (size_t)tmax * 256 * sizeof(float), hipMemcpyHostToDevice));
    ctx->tmax = tmax;
    ++ctx->table_gen;
  });
}

int dmx_model_cfg_num_keys(const dmx_model_config* cfg) {
  if (cfg == nullptr) return -1;
  int n = -1;
  if (guarded([&] { n = (int)model_keys(to_cfg(*cfg)).size(); }) != DMX_OK) return -1;
  return n;
}

int dmx_model_num_keys(int kind, int in_ch, int remove_deep_conv) {
  const dmx_model_config c = default_cfg(kind, in_ch, remove_deep_conv);
  return dmx_model_cfg_num_keys(&c);
}

int dmx_model_key(int kind, int in_ch, int remove_deep_conv, int index, char* name_out, int name_cap,
                  int64_t* shape_out, int* ndim_out) {
  const dmx_model_config c = default_cfg(kind, in_ch, remove_deep_conv);
  return dmx_model_cfg_key(&c, index, name_out, name_cap, shape_out, ndim_out);
}

int dmx_model_cfg_key(const dmx_model_config* cfg, int index, char* name_out, int name_cap, int64_t* shape_out,
                      int* ndim_out) {
  return guarded([&] {
    REQUIRE(cfg != nullptr, "null config");
    Keys k = model_keys(to_cfg(*cfg));
    REQUIRE(index >= 0 && index < (int)k.size(), "key index out of range");
    REQUIRE(name_out && name_cap > (int)k[index].name.size(), "name buffer too small");
    std::strcpy(name_out, k[index].name.c_str());
    if (ndim_out) *ndim_out = (int)k[index].shape.size();
    if (shape_out)
      for (size_t i = 0; i < k[index].shape.size() && i < 4; ++i) shape_out[i] = k[index].shape[i];
  });
}

int dmx_model_create_cfg(dmx_ctx* ctx, const dmx_model_config* cfg, dmx_model** out) {
  return guarded([&] {
    REQUIRE(ctx && cfg && out, "null argument");
    const ModelCfg c = to_cfg(*cfg);
    auto* m = new dmx_model();
    m->ctx = ctx;
    m->cfg = c;
    m->kind = c.kind;
    m->in_ch = c.in_ch;
    m->deep = c.deep;
    m->keys = model_keys(c);
    *out = m;
  });
}

int dmx_model_create(dmx_ctx* ctx, int kind, int in_ch, int remove_deep_conv, dmx_model** out) {
  const dmx_model_config c = default_cfg(kind, in_ch, remove_deep_conv);
  return dmx_model_create_cfg(ctx, &c, out);
}

int dmx_model_destroy(dmx_model* m) {
  return guarded([&] {
    if (!m) return;
    drop_graph(m);
    for (void* p : m->owned) (void)hipFree(p);
    if (m->job_tables) (void)hipFree(m->job_tables);
    if (m->split_table) (void)hipFree(m->split_table);
    if (m->ws_mem) (void)hipFree(m->ws_mem);
    if (m->tws_mem) (void)hipFree(m->tws_mem);
    if (m->bws_mem) (void)hipFree(m->bws_mem);
    delete m->tape;
    delete m;
  });
}

int dmx_model_set_tensor(dmx_model* m, const char* name, const float* dev_ptr, const int64_t* shape, int ndim) {
  return guarded([&] {
    REQUIRE(m && name && dev_ptr && (ndim == 0 || shape), "null argument");
    REQUIRE(ndim >= 0 && ndim <= 4, "ndim must be <= 4");
    std::vector<int64_t> s(shape, shape + ndim);
    bool known = false;
    for (auto& k : m->keys)
      if (k.name == name) {
        known = true;
        if (k.shape != s) throw Error(DMX_E_ARG, std::string("shape mismatch for '") + name + "'");
      }
    if (!known) throw Error(DMX_E_ARG, std::string("unexpected key '") + name + "'");
    m->inputs[name] = {dev_ptr, s};
  });
}

int dmx_model_finalize(dmx_model* m, void* stream) {
  return guarded([&] {
    REQUIRE(m, "null model");
    finalize_model(m, (hipStream_t)stream);
  });
}

int64_t dmx_model_workspace_bytes(const dmx_model* m) { return m ? (int64_t)m->ws_cap : -1; }

int dmx_model_refresh(dmx_model* m, void* stream) {
  return guarded([&] {
    REQUIRE(m != nullptr, "null model");
    refresh_model(m, (hipStream_t)stream);
  });
}

int dmx_train_forward(dmx_model* m, const float* x, const int64_t* t, const int64_t* y, const float* vals,
                      const float* mask, int n, int h, int w, float* eps, float* geom, int64_t* tape_id,
                      void* stream) {
  return guarded([&] {
    REQUIRE(m != nullptr && tape_id != nullptr, "null argument");
    check_train(m, n, h, w);
    REQUIRE(x && t && y && eps, "null tensor");
    REQUIRE((vals == nullptr) == (mask == nullptr), "vals and mask must be given together");
    REQUIRE(geom == nullptr || m->kind == DMX_UNET_COND_GEOM, "geom output only for UnetCondWithGeomHead");
    hipStream_t st = (hipStream_t)stream;
    ensure_train(m, st);
    if (m->tape == nullptr) m->tape = new Tape();
    Tape& T = *m->tape;
    T.id = 0;  // invalid until the forward below has been enqueued
    TrainArgs a{x, t, y, vals, mask, n, h, w, eps, geom};
    with_fp32(m, [&] {
      run_arena(m, st, m->tws, m->tws_mem, m->tws_cap, [&](Run& R) { train_fwd_body(R, T, a); });
    });
    T.id = ++m->tape_id;
    *tape_id = T.id;
  });
}

int dmx_train_backward(dmx_model* m, int64_t tape_id, const float* d_eps, const float* d_geom, float* const* grads,
                       int n_grads, void* stream) {
  return guarded([&] {
    REQUIRE(m != nullptr && grads != nullptr, "null argument");
    REQUIRE(m->tape != nullptr && m->tape->id != 0, "no training forward recorded (dmx_train_forward)");
    REQUIRE(tape_id == m->tape->id,
            "stale tape: another dmx_train_forward ran after the one this backward belongs to");
    REQUIRE(n_grads == (int)m->keys.size(), "grads must hold one pointer per state_dict key");
    GradMap G;
    for (int i = 0; i < n_grads; ++i) G.g[m->keys[i].name] = grads[i];
    hipStream_t st = (hipStream_t)stream;
    with_fp32(m, [&] {
      run_arena(m, st, m->bws, m->bws_mem, m->bws_cap, [&](Run& R) { train_bwd_body(R, *m->tape, G, d_eps, d_geom); });
    });
  });
}

int dmx_attn_core_backward(const float* qkv, const float* o, const float* dout, float* dqkv, int n, int L, int C,
                           void* stream) {
  return guarded([&] {
    REQUIRE(qkv && o && dout && dqkv, "null tensor");
    REQUIRE(n >= 1 && L >= 1 && (C == 64 || C == 128 || C == 256), "attention backward: n, L >= 1, C in {64, 128, 256}");
    hipStream_t st = (hipStream_t)stream;
    float* sbuf = nullptr;
    HIPCHK(hipMallocAsync(reinterpret_cast<void**>(&sbuf), (size_t)n * 4 * L * 3 * sizeof(float), st));
    attn_core_bwd_launch(qkv, o, dout, dqkv, sbuf, n, L, C, false, st);
    HIPCHK(hipFreeAsync(sbuf, st));
  });
}

int dmx_model_set_precision(dmx_model* m, int prec) {
  return guarded([&] {
    REQUIRE(m != nullptr, "null model");
    REQUIRE(prec >= 0 && prec <= 2, "precision must be 0 (fp32 MFMA), 1 (fp16x3 split) or 2 (fp16, config 4)");
    if (m->prec != prec) drop_graph(m);
    m->prec = prec;
  });
}

int dmx_model_get_precision(const dmx_model* m) { return m ? m->prec : -1; }

int dmx_model_range_check(dmx_model* m, int reset, int* flagged, void* stream) {
  return guarded([&] {
    REQUIRE(m != nullptr && flagged != nullptr, "null argument");
    if (!m->finalized) throw Error(DMX_E_STATE, "model weights not finalized");
    hipStream_t st = (hipStream_t)stream;
    int v = 0;
    HIPCHK(hipMemcpyAsync(&v, m->range_flag, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *flagged = v;
    if (reset) HIPCHK(hipMemsetAsync(m->range_flag, 0, sizeof(int), st));
  });
}

int dmx_debug_enable(dmx_model* m, int on) {
  return guarded([&] {
    REQUIRE(m != nullptr, "null model");
    m->debug = on != 0;
    m->taps.clear();
  });
}

int dmx_debug_num_taps(const dmx_model* m) { return m ? (int)m->taps.size() : -1; }

int dmx_debug_tap(dmx_model* m, int i, char* name_out, int cap, int64_t* count_out, float* dst, void* stream) {
  return guarded([&] {
    REQUIRE(m && i >= 0 && i < (int)m->taps.size(), "bad tap index");
    auto& t = m->taps[i];
    REQUIRE(name_out && cap > (int)t.first.size(), "name buffer too small");
    std::strcpy(name_out, t.first.c_str());
    if (count_out) *count_out = (int64_t)t.second.second;
    if (dst)
      HIPCHK(hipMemcpyAsync(dst, t.second.first, t.second.second * sizeof(float), hipMemcpyDeviceToDevice,
                            (hipStream_t)stream));
  });
}

int dmx_unet_forward(dmx_model* m, const float* x, const int64_t* t, const int64_t* y, const float* vals,
                     const float* mask, float* eps, float* geom, int n, int h, int w, void* stream) {
  return guarded([&] {
    REQUIRE(m != nullptr, "null model");
    check_shapes(m, n, h, w);
    REQUIRE(x && t && eps, "null tensor");
    if (m->kind != DMX_UNET) REQUIRE(y != nullptr, "conditional U-Net needs y");
    REQUIRE((vals == nullptr) == (mask == nullptr), "vals and mask must be given together");
    REQUIRE(geom == nullptr || m->kind == DMX_UNET_COND_GEOM, "geom output only for UnetCondWithGeomHead");
    hipStream_t st = (hipStream_t)stream;
    ensure_planes(m, st);
    m->taps.clear();
    run_planned(m, st, [&](Run& R) {
      FwdIn in{x, n, t, 1, y, 0, 0, vals, mask, n};
      float* feat = unet_trunk(R, in, n, h, w);
      if (R.plan) return;
      dim3 grid(cdiv(h * w, 256), n);
      out_head_kernel<<<grid, 256, 0, st>>>(feat, m->out_w, m->out_b, eps, m->in_ch, h * w, m->range_flag);
      HIPCHK(hipGetLastError());
      if (geom) {
        geom_head_kernel<<<n, 256, (64 + m->cfg.ghid) * sizeof(float), st>>>(feat, h * w, m->gw0, m->gb0, m->gw2, m->gb2,
                                                                             m->cfg.ghid, m->cfg.gdim, geom);
        HIPCHK(hipGetLastError());
      }
    });
  });
}

int dmx_step(dmx_model* m, const dmx_step_args* a, void* stream) {
  return guarded([&] {
    REQUIRE(m != nullptr, "null model");
    validate_step(m, a);
    ensure_planes(m, (hipStream_t)stream);
    run_planned(m, (hipStream_t)stream, [&](Run& R) { step_body(R, *a); });
  });
}

static constexpr int kGraphSteps = 8;

int dmx_sample_loop(dmx_model* m, const dmx_step_args* a, int steps, int use_graph, void* stream) {
  return guarded([&] {
    REQUIRE(m != nullptr, "null model");
    validate_step(m, a);
    REQUIRE(a->x_in == a->x_out, "sample loop runs in place (x_in == x_out)");
    REQUIRE(a->t_stride == 0, "sample loop needs a device scalar t (t_stride 0)");
    REQUIRE(a->noise == nullptr, "sample loop draws on-device Philox noise (noise must be NULL)");
    REQUIRE(steps >= 0, "steps must be >= 0");
    hipStream_t st = (hipStream_t)stream;
    ensure_planes(m, st);
    int64_t* tdev = const_cast<int64_t*>(a->t);
    if (!use_graph) {
      for (int i = 0; i < steps; ++i) {
        run_planned(m, st, [&](Run& R) { step_body(R, *a); });
        decrement_t_kernel<<<1, 64, 0, st>>>(tdev);
        HIPCHK(hipGetLastError());
      }
      return;
    }
    GraphKey key;
    std::memset(&key, 0, sizeof(key));
    std::memcpy(&key.a, a, sizeof(dmx_step_args));
    key.table_gen = m->ctx->table_gen;
    if (!(m->has_graph && key == m->gkey)) {
      drop_graph(m);
      // plan + allocate outside capture, then capture the real launches
      m->ws.base = nullptr;
      m->ws.off = 0;
      m->ws.plan = true;
      {
        Run P{m, st, true, m->ws};
        step_body(P, *a);
      }
      ensure_ws(m);
      poison(m->ws_mem, m->ws.off, st);
      m->ws.base = static_cast<char*>(m->ws_mem);
      m->ws.off = 0;
      m->ws.plan = false;
      HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      try {
        Run R{m, st, false, m->ws};
        step_body(R, *a);
        decrement_t_kernel<<<1, 64, 0, st>>>(tdev);
      } catch (...) {
        hipGraph_t g;
        (void)hipStreamEndCapture(st, &g);
        if (g) (void)hipGraphDestroy(g);
        throw;
      }
      HIPCHK(hipStreamEndCapture(st, &m->graph));
      HIPCHK(hipGraphInstantiate(&m->gexec, m->graph, nullptr, nullptr, 0));
      m->has_graph = true;  // owns gexec / graph from here (drop_graph frees them on any failure below)
      // kGraphSteps consecutive steps in one graph: the gap between two graph launches (≈9 µs of
      // idle GPU per step in the replay trace) is paid once per kGraphSteps steps.  Inside it, t
      // alternates between the caller's scalar and a scratch scalar: step k reads one and its
      // embedding kernel stores t - 1 in the other (no one-thread decrement launch per step; an even
      // kGraphSteps ends in the caller's scalar).  The noise is keyed by (seed, t, sample), so the
      // captured steps compute what kGraphSteps replays of the one-step graph compute.
      static_assert(kGraphSteps % 2 == 0, "t ping-pong must end in the caller's buffer");
      int64_t* tscr = m->t_scratch;
      HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      try {
        for (int k = 0; k < kGraphSteps; ++k) {
          m->ws.off = 0;
          Run R{m, st, false, m->ws};
          dmx_step_args ak = *a;
          ak.t = (k & 1) ? tscr : tdev;
          step_body(R, ak, (k & 1) ? tdev : tscr, k > 0);  // cond MLP rows from step 0 of the graph
        }
      } catch (...) {
        hipGraph_t g;
        (void)hipStreamEndCapture(st, &g);
        if (g) (void)hipGraphDestroy(g);
        drop_graph(m);
        throw;
      }
      const hipError_t ec = hipStreamEndCapture(st, &m->graph_k);
      const hipError_t ei = ec == hipSuccess ? hipGraphInstantiate(&m->gexec_k, m->graph_k, nullptr, nullptr, 0) : ec;
      if (ei != hipSuccess) {  // never leave a key that claims a graph pair without the 8-step exec
        drop_graph(m);
        HIPCHK(ei);
      }
      m->gkey = key;  // only once both graphs are instantiated
    }
    int i = 0;
    for (; i + kGraphSteps <= steps; i += kGraphSteps) HIPCHK(hipGraphLaunch(m->gexec_k, st));
    for (; i < steps; ++i) HIPCHK(hipGraphLaunch(m->gexec, st));
  });
}

int dmx_step_profile(dmx_model* m, const dmx_step_args* a, dmx_kernel_record* recs, int cap, int* n_out,
                     void* stream) {
  return guarded([&] {
    REQUIRE(m != nullptr && recs != nullptr && n_out != nullptr, "null argument");
    validate_step(m, a);
    hipStream_t st = (hipStream_t)stream;
    ensure_planes(m, st);
    Prof prof;
    m->ws.base = nullptr;
    m->ws.off = 0;
    m->ws.plan = true;
    {
      Run P{m, st, true, m->ws};
      step_body(P, *a);
    }
    ensure_ws(m);
    m->ws.base = static_cast<char*>(m->ws_mem);
    m->ws.off = 0;
    m->ws.plan = false;
    Run R{m, st, false, m->ws, &prof};
    step_body(R, *a);
    HIPCHK(hipStreamSynchronize(st));
    int n = 0;
    for (auto& r : prof.recs) {
      if (n >= cap) break;
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, r.e0, r.e1));
      std::memset(&recs[n], 0, sizeof(recs[n]));
      std::snprintf(recs[n].kernel, sizeof recs[n].kernel, "%s", r.kernel.c_str());
      std::snprintf(recs[n].layer, sizeof recs[n].layer, "%s", r.layer.c_str());
      recs[n].flops = r.flops;
      recs[n].bytes = r.bytes;
      recs[n].ms = ms;
      ++n;
    }
    *n_out = n;
  });
}

int dmx_ddpm_update(const float* x, float* x_out, const float* eu, const float* ec, float guidance,
                    const int64_t* t, int t_stride, const float* c1, const float* c2, const float* sd, int T,
                    const float* noise, uint64_t seed, int64_t sample_offset, int n, int c, int h, int w,
                    void* stream) {
  return guarded([&] {
    REQUIRE(x && x_out && eu && t && c1 && c2 && sd, "null tensor");
    REQUIRE(n >= 1 && c >= 1 && c <= 4 && h >= 1 && w >= 1 && T >= 1, "bad shape");
    StepTailParams p;
    std::memset(&p, 0, sizeof(p));
    p.Co = c;
    p.B = n;
    p.HW = h * w;
    p.cfg = ec != nullptr ? 1 : 0;
    p.guidance = guidance;
    p.eps_u = eu;
    p.eps_c = ec;
    p.x = x;
    p.x_out = x_out;
    p.t = t;
    p.t_stride = t_stride;
    p.tmax = T;
    p.c1 = c1;
    p.c2 = c2;
    p.sd = sd;
    p.noise = noise;
    p.seed = seed;
    p.sample_offset = sample_offset;
    dim3 grid(cdiv(p.HW, 256), n);
    step_tail_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(p);
    HIPCHK(hipGetLastError());
  });
}

int dmx_vae_decode(dmx_model* m, const float* z, float* img, uint8_t* u8, int n, int h, int w, void* stream) {
  return guarded([&] {
    REQUIRE(m != nullptr, "null model");
    if (!m->finalized) throw Error(DMX_E_STATE, "model weights not finalized");
    REQUIRE(m->kind == DMX_VAE, "not a VAE model");
    REQUIRE(z && (img || u8), "null tensor");
    REQUIRE(n >= 1 && h >= 1 && w >= 1, "bad shape");
    const int chunk = 16;  // bounds workspace (the reference decodes in chunks of 4, diff.py:353)
    hipStream_t st = (hipStream_t)stream;
    ensure_planes(m, st);
    for (int s = 0; s < n; s += chunk) {
      const int b = std::min(chunk, n - s);
      run_planned(m, st, [&](Run& R) {
        vae_body(R, z + (size_t)s * 4 * h * w, img ? img + (size_t)s * 3 * 64 * h * w : nullptr,
                 u8 ? u8 + (size_t)s * 64 * h * w * 3 : nullptr, b, h, w);
      });
    }
  });
}

int dmx_latent_frames_u8(const float* z, uint8_t* out, int n, int c, int h, int w, void* stream) {
  return guarded([&] {
    REQUIRE(z && out, "null tensor");
    REQUIRE(n >= 1 && c >= 1 && h >= 1 && w >= 1, "bad shape");
    latent_frames_kernel<<<n * c, 256, 0, (hipStream_t)stream>>>(z, out, h * w);
    HIPCHK(hipGetLastError());
  });
}

int dmx_eval_metrics(const uint8_t* gt, const uint8_t* pred, int n, int h, int w, int gray, int threshold, int invert,
                     double sigma, int* workspace, double* out, void* stream) {
  return guarded([&] {
    REQUIRE(gt && pred && workspace && out, "null tensor");
    REQUIRE(n >= 1 && h >= 1 && w >= 1 && h <= 16384 && w <= 16384, "bad shape (1 <= h, w <= 16384)");
    REQUIRE((size_t)h * w < ((size_t)1 << 31) && (size_t)h * h + (size_t)w * w < ((size_t)1 << 30), "image too large");
    EvalParams p{gt, pred, h, w, gray, threshold, invert, sigma, workspace, out};
    eval_metrics_kernel<<<n, 256, 0, (hipStream_t)stream>>>(p);
    HIPCHK(hipGetLastError());
  });
}

int dmx_vae_encode(dmx_model* m, const float* x, const float* eps, float* z, float* kl, int n, int h, int w,
                   void* stream) {
  return guarded([&] {
    REQUIRE(m != nullptr, "null model");
    if (!m->finalized) throw Error(DMX_E_STATE, "model weights not finalized");
    REQUIRE(m->kind == DMX_VAE, "not a VAE model");
    REQUIRE(x && eps && z && kl, "null tensor");
    REQUIRE(n >= 1 && h >= 8 && w >= 8 && h % 8 == 0 && w % 8 == 0, "image sides must be multiples of 8");
    const int chunk = 16;  // bounds workspace
    const int hl = h / 8, wl = w / 8;
    hipStream_t st = (hipStream_t)stream;
    ensure_planes(m, st);
    for (int s = 0; s < n; s += chunk) {
      const int b = std::min(chunk, n - s);
      run_planned(m, st, [&](Run& R) {
        vae_enc_body(R, x + (size_t)s * 3 * h * w, eps + (size_t)s * 4 * hl * wl, z + (size_t)s * 4 * hl * wl,
                     kl + s, b, h, w);
      });
    }
  });
}

}  // extern "C"
