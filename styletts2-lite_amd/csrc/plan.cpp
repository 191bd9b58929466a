// Model plans (HiFi-GAN / iSTFTNet decoders, F0/N conv stacks, style encoder) and the
// C-ABI declared in include/stts2.h.  A plan is built from the constructor arguments of the
// reference module, names every parameter exactly like the reference state dict, packs the
// weights (weight-norm fold + MFMA layout) into a caller buffer, and strings the gfx950
// kernels together for one forward.  All launches go to the caller's stream; the workspace
// is carved by a bump allocator whose dry run gives stts_workspace_bytes().
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/stts2.h"
#include "common.h"
#include "kernels.h"

namespace {

constexpr size_t ALIGN = 256;
inline size_t rup(size_t x, size_t a) { return (x + a - 1) / a * a; }
inline int rup8(int x) { return (x + 7) & ~7; }

// ----------------------------------------------------------------------- profiling
struct Prof {
  bool on = false;
  std::vector<hipEvent_t> ev;  // pairs
  size_t used = 0;
  long long launches = 0;
  double flops = 0, bytes = 0;
  struct Rec { int shape[8]; double flops, bytes; };
  std::vector<Rec> rec;  // one per timed launch, in launch order
} g_prof;

// ----------------------------------------------------------------------- parameters
struct Params {
  std::vector<std::string> names;
  std::vector<long long> numel;
  std::vector<const float*> ptr;
  int add(const std::string& n, long long k) {
    names.push_back(n);
    numel.push_back(k);
    ptr.push_back(nullptr);
    return (int)names.size() - 1;
  }
  const float* operator[](int i) const { return i < 0 ? nullptr : ptr[i]; }
};

// A convolution whose weights are packed for conv1d_igemm.
struct WConv {
  int v = -1, g = -1, bias = -1;
  int Cin = 0, Cout = 0, K = 0, transposed = 0, u = 1;
  int reframe = 0;  // > 0: a Conv1d(1, Cout, 2S, stride S) packed as a 2-tap conv over S-sample frames
  // pack-time prep (Vocos): rows scaled by parameter `rs` (layer scale), or only `src_rows` < Cout rows
  // in the parameter (the rest packed as zero columns); the bias then lives folded / padded in aux
  int rs = -1, src_rows = 0;
  size_t bias_aux = 0;
  bool aux_bias = false;
  size_t off[ST_NDTYPES] = {0, 0, 0};
  // fold > 1: a stride-`fold` conv (padding fpad0) packed as the stride-1 conv over phase-folded frames
  // (fold consecutive input rows side by side): fold Cin channels, fK taps, padding fpad (k_fold_w)
  int fold = 0, fpad0 = 0, fK = 0, fpad = 0;
  int taps() const { return fold ? fK : (transposed ? (K + u - 1) / u : K); }
  int N() const { return transposed ? u * Cout : Cout; }
  int pCin() const { return fold ? fold * Cin : Cin; }
};

// the stride-1 form of a stride-st conv (K taps, padding pad): input row st q + t - pad = st (q + s') + ph
void set_fold(WConv& c, int st, int pad) {
  int smin = 1 << 30, smax = -(1 << 30);
  for (int t = 0; t < c.K; ++t) {
    const int j = t - pad;
    const int sq = j >= 0 ? j / st : -((-j + st - 1) / st);  // floor(j / st)
    smin = std::min(smin, sq);
    smax = std::max(smax, sq);
  }
  c.fold = st;
  c.fpad0 = pad;
  c.fK = smax - smin + 1;
  c.fpad = -smin;
}

struct WAdaIN {
  int w = -1, b = -1, C = 0, hoff = 0;
};

struct ResBlock1 {  // AdaINResBlock1 (hifigan.py:26-80)
  int C = 0, K = 0, dil[3] = {1, 3, 5};
  WConv c1[3], c2[3];
  WAdaIN a1[3], a2[3];
  int al1[3], al2[3];
};

struct AdainBlk {  // AdainResBlk1d (hifigan.py:359-403)
  int cin = 0, cout = 0;
  bool up = false, learned = false;
  WConv conv1, conv2, sc;
  WAdaIN n1, n2;
  int pool_v = -1, pool_g = -1, pool_b = -1;
  size_t pool_off = 0;  // folded fp32 [cin][3] in the aux area
};

struct Small {  // weight-norm conv folded to fp32 for a VALU kernel
  int v = -1, g = -1, bias = -1;
  long long rows = 0, inner = 0;
  size_t off = 0;
};

}  // namespace

struct stts_model {
  int kind = 0;
  Params P;
  // small-batch decoder: the stage's resblocks 1.. on side streams (decoder_forward), created on first use
  hipStream_t side[4] = {};
  hipEvent_t ev_fork = nullptr, ev_join[4] = {}, ev_fork2 = nullptr, ev_noise[8] = {};
  // the side streams and events are per model: concurrent forwards of one model (with their own workspaces and
  // streams) take turns through the forks and joins, so each wait sees its own forward's record
  std::mutex branch_mu;
  stts_model() = default;
  stts_model(const stts_model&) = delete;
  stts_model& operator=(const stts_model&) = delete;
  ~stts_model() {
    for (auto& s : side)
      if (s) (void)hipStreamDestroy(s);
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    if (ev_fork2) (void)hipEventDestroy(ev_fork2);
    for (auto& e : ev_join)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : ev_noise)
      if (e) (void)hipEventDestroy(e);
  }
  // -------- decoder config
  int dim_in = 512, style_dim = 128, init_ch = 512, n_fft = 0, hop = 0;
  std::vector<int> rates, kernels, rbk;
  std::vector<std::vector<int>> rbd;
  // -------- decoder layers
  AdainBlk encode, decode[4];
  Small F0_conv, N_conv;
  WConv asr_res;
  int l_lin_w = -1, l_lin_b = -1;
  std::vector<int> nc_w, nc_b;      // hifigan noise_convs (Cin=1): raw [C][K] (VALU kernel), -1 if nc_mm
  std::vector<WConv> nc_mm;         // hifigan noise_convs with K >= 16: 2-tap MFMA conv over S-sample frames
  std::vector<WConv> nc_conv;       // istftnet noise_convs (Cin=n_fft+2): igemm
  std::vector<WConv> ups;
  std::vector<ResBlock1> noise_res, resblocks;
  std::vector<int> alphas;
  WConv conv_post;
  int stft_fr = -1, stft_fi = -1, stft_br = -1, stft_bi = -1;
  // -------- Vocos generator (Modules/vocos.py:108-162, ISTFTHead :248-296)
  bool pwn = false;  // weight norm as torch.nn.utils.parametrizations (original0 = g, original1 = v)
  int vc_inter = 0, vc_layers = 0;
  struct CNX {
    int dw_w = -1, dw_b = -1, gamma = -1;
    WAdaIN norm;
    WConv pw1, pw2;
  };
  std::vector<CNX> cnx;
  int ln_w = -1, ln_b = -1, vwin = -1;
  WConv vhead;  // -------- F0N
  int d_hid = 512;
  AdainBlk f0blk[3], nblk[3];
  WConv f0_proj, n_proj;
  // -------- style encoder (models.py:125-150)
  struct SEBlk {
    int cin = 0, cout = 0;
    bool learned = false;
    WConv conv1, conv2, sc;
    int dw_w = -1, dw_b = -1;
  } se_blk[4];
  WConv se_conv0, se_last;
  int se_lin_w = -1, se_lin_b = -1, se_dim = 0;
  // -------- MultiPeriodDiscriminator (Modules/discriminators.py:96-156)
  struct DiscP {
    int period = 0;
    WConv convs[5], post;
  };
  std::vector<DiscP> mpd;
  // -------- MultiResSpecDiscriminator (Modules/discriminators.py:29-94)
  struct DiscS {
    int n_fft = 0, hop = 0, win = 0;
    WConv convs[5], out;
  };
  std::vector<DiscS> msd;
  // -------- AdaIN projections (all AdaIN layers share one GEMV: H = s @ Wt + b)
  std::vector<WAdaIN*> adains;
  int Htot = 0;
  size_t wt_off = 0, bcat_off = 0;  // fp32 Wt [style_dim][Htot], bias [Htot] in the aux area
  // -------- packing
  std::vector<WConv*> convs;
  std::vector<Small*> smalls;
  std::vector<AdainBlk*> pools;
  size_t conv_bytes[ST_NDTYPES] = {0, 0, 0};
  size_t aux_off[ST_NDTYPES] = {0, 0, 0}, aux_bytes = 0, scratch_off[ST_NDTYPES] = {0, 0, 0}, scratch_bytes = 0;
  size_t total_bytes[ST_NDTYPES] = {0, 0, 0};
  const char* packed[ST_NDTYPES] = {nullptr, nullptr, nullptr};
};

namespace {

using Model = stts_model;

// ----------------------------------------------------------------------- builders
void add_wconv(Model& m, WConv& c, const std::string& p, int cin, int cout, int k, bool wn, bool bias,
               int transposed = 0, int u = 1, int groups = 1) {
  c.Cin = cin;
  c.Cout = cout;
  c.K = k;
  c.transposed = transposed;
  c.u = u;
  if (bias) c.bias = m.P.add(p + ".bias", cout);
  if (wn) {
    c.g = m.P.add(p + (m.pwn ? ".parametrizations.weight.original0" : ".weight_g"), transposed ? cin : cout);
    c.v = m.P.add(p + (m.pwn ? ".parametrizations.weight.original1" : ".weight_v"), (long long)cin * cout / groups * k);
  } else {
    c.v = m.P.add(p + ".weight", (long long)cin * cout / groups * k);
  }
  m.convs.push_back(&c);
}

void add_adain(Model& m, WAdaIN& a, const std::string& p, int C) {
  a.C = C;
  a.w = m.P.add(p + ".fc.weight", (long long)2 * C * m.style_dim);
  a.b = m.P.add(p + ".fc.bias", 2 * C);
  m.adains.push_back(&a);
}

void add_resblock1(Model& m, ResBlock1& r, const std::string& p, int C, int K, const int* dil) {
  r.C = C;
  r.K = K;
  for (int j = 0; j < 3; ++j) r.dil[j] = dil[j];
  for (int j = 0; j < 3; ++j) add_wconv(m, r.c1[j], p + ".convs1." + std::to_string(j), C, C, K, true, true);
  for (int j = 0; j < 3; ++j) add_wconv(m, r.c2[j], p + ".convs2." + std::to_string(j), C, C, K, true, true);
  for (int j = 0; j < 3; ++j) add_adain(m, r.a1[j], p + ".adain1." + std::to_string(j), C);
  for (int j = 0; j < 3; ++j) add_adain(m, r.a2[j], p + ".adain2." + std::to_string(j), C);
  for (int j = 0; j < 3; ++j) r.al1[j] = m.P.add(p + ".alpha1." + std::to_string(j), C);
  for (int j = 0; j < 3; ++j) r.al2[j] = m.P.add(p + ".alpha2." + std::to_string(j), C);
}

void add_adainblk(Model& m, AdainBlk& b, const std::string& p, int cin, int cout, bool up) {
  b.cin = cin;
  b.cout = cout;
  b.up = up;
  b.learned = cin != cout;
  add_wconv(m, b.conv1, p + ".conv1", cin, cout, 3, true, true);
  add_wconv(m, b.conv2, p + ".conv2", cout, cout, 3, true, true);
  add_adain(m, b.n1, p + ".norm1", cin);
  add_adain(m, b.n2, p + ".norm2", cout);
  if (b.learned) add_wconv(m, b.sc, p + ".conv1x1", cin, cout, 1, true, false);
  if (up) {
    b.pool_b = m.P.add(p + ".pool.bias", cin);
    b.pool_g = m.P.add(p + (m.pwn ? ".pool.parametrizations.weight.original0" : ".pool.weight_g"), cin);
    b.pool_v = m.P.add(p + (m.pwn ? ".pool.parametrizations.weight.original1" : ".pool.weight_v"), (long long)cin * 3);
    m.pools.push_back(&b);
  }
}

void add_small_wn(Model& m, Small& s, const std::string& p, long long rows, long long inner) {
  s.rows = rows;
  s.inner = inner;
  s.bias = m.P.add(p + ".bias", rows);
  s.g = m.P.add(p + (m.pwn ? ".parametrizations.weight.original0" : ".weight_g"), rows);
  s.v = m.P.add(p + (m.pwn ? ".parametrizations.weight.original1" : ".weight_v"), rows * inner);
  m.smalls.push_back(&s);
}

// decoder front-end (hifigan.py:427-440 == istftnet.py:673-686 == vocos.py:370-390)
void add_frontend(Model& m) {
  add_adainblk(m, m.encode, "encode", m.dim_in + 2, 1024, false);
  for (int k = 0; k < 4; ++k)
    add_adainblk(m, m.decode[k], "decode." + std::to_string(k), 1024 + 2 + 64, k == 3 ? 512 : 1024, k == 3);
  add_small_wn(m, m.F0_conv, "F0_conv", 1, 3);
  add_small_wn(m, m.N_conv, "N_conv", 1, 3);
  add_wconv(m, m.asr_res, "asr_res.0", m.dim_in, 64, 1, true, true);
}

// Vocos Decoder (Modules/vocos.py:364-390): cfg = dim_in, style_dim, intermediate_dim, num_layers,
// n_fft, hop.  The generator's dim is dim_in and its input is decode.3's 512 channels, so the
// reference itself only runs with dim_in = 512.
int build_vocos(Model& m, const int* cfg, int n) {
  if (n != 6) return ST_EINVAL;
  m.dim_in = cfg[0];
  m.style_dim = cfg[1];
  m.vc_inter = cfg[2];
  m.vc_layers = cfg[3];
  m.n_fft = cfg[4];
  m.hop = cfg[5];
  if (m.dim_in != 512 || m.style_dim <= 0 || m.vc_inter <= 0 || m.vc_inter % 32 || m.vc_layers <= 0 ||
      m.vc_layers > 64 || m.hop <= 0 || m.hop > m.n_fft || (m.n_fft - m.hop) / 2 <= 0)
    return ST_EINVAL;
  int n1 = 0, n2 = 0;
  if (st_istft_factor(m.n_fft, &n1, &n2) != ST_OK) return ST_EINVAL;
  m.pwn = true;
  add_frontend(m);
  const int d = m.dim_in;
  m.cnx.resize(m.vc_layers);  // sized once: add_wconv / add_adain keep pointers into it
  for (int i = 0; i < m.vc_layers; ++i) {
    auto& b = m.cnx[i];
    const std::string p = "generator.convnext." + std::to_string(i);
    b.dw_w = m.P.add(p + ".dwconv.weight", (long long)d * 7);
    b.dw_b = m.P.add(p + ".dwconv.bias", d);
    add_adain(m, b.norm, p + ".norm", d);
    add_wconv(m, b.pw1, p + ".pwconv1", d, m.vc_inter, 1, false, true);  // nn.Linear == [Cout][Cin][1]
    add_wconv(m, b.pw2, p + ".pwconv2", m.vc_inter, d, 1, false, true);
    b.gamma = m.P.add(p + ".gamma", d);
    b.pw2.rs = b.gamma;  // gamma * (W x + b) folded into the packed weights and bias
    b.pw2.aux_bias = true;
  }
  m.ln_w = m.P.add("generator.final_layer_norm.weight", d);
  m.ln_b = m.P.add("generator.final_layer_norm.bias", d);
  const int nout = 2 * (m.n_fft / 2 + 1);
  add_wconv(m, m.vhead, "generator.stft.out", d, nout, 1, false, true);
  m.vhead.src_rows = nout;  // columns padded to the MFMA 16-column multiple (the wide epilogue)
  m.vhead.Cout = (nout + 15) & ~15;
  m.vhead.aux_bias = true;
  m.vwin = m.P.add("generator.stft.istft.window", m.n_fft);
  return ST_OK;
}

int build_decoder(Model& m, const int* cfg, int n) {
  int i = 0;
  auto take = [&](int& dst) -> bool {
    if (i >= n) return false;
    dst = cfg[i++];
    return true;
  };
  int nup = 0, nrb = 0;
  if (!take(m.dim_in) || !take(m.style_dim) || !take(m.init_ch) || !take(nup) || nup <= 0 || nup > 8) return ST_EINVAL;
  m.rates.resize(nup);
  m.kernels.resize(nup);
  for (auto& r : m.rates)
    if (!take(r) || r <= 0) return ST_EINVAL;
  for (auto& k : m.kernels)
    if (!take(k) || k <= 0) return ST_EINVAL;
  if (!take(nrb) || nrb <= 0 || nrb > 8) return ST_EINVAL;
  m.rbk.resize(nrb);
  m.rbd.assign(nrb, std::vector<int>(3));
  for (auto& k : m.rbk)
    if (!take(k) || k <= 0 || k % 2 == 0) return ST_EINVAL;
  for (auto& d : m.rbd)
    for (auto& x : d)
      if (!take(x) || x <= 0) return ST_EINVAL;
  if (m.kind == STTS_KIND_ISTFTNET) {
    if (!take(m.n_fft) || !take(m.hop) || m.n_fft <= 0 || m.hop <= 0) return ST_EINVAL;
  }
  if (i != n) return ST_EINVAL;
  if (m.init_ch != 512) return ST_EINVAL;  // decode.3 emits 512 channels (hifigan.py:432)
  const bool ist = m.kind == STTS_KIND_ISTFTNET;
  add_frontend(m);
  // generator (hifigan.py:272-319 / istftnet.py:494-540)
  m.l_lin_w = m.P.add("generator.m_source.l_linear.weight", 9);
  m.l_lin_b = m.P.add("generator.m_source.l_linear.bias", 1);
  m.ups.resize(nup);
  m.noise_res.resize(nup);
  m.resblocks.resize((size_t)nup * nrb);
  if (ist) m.nc_conv.resize(nup);
  else m.nc_mm.resize(nup);
  static const int d135[3] = {1, 3, 5};
  for (int s = 0; s < nup; ++s) {
    const int u = m.rates[s], k = m.kernels[s];
    const int cin = m.init_ch >> s, c = m.init_ch >> (s + 1);
    const std::string gp = "generator.";
    add_wconv(m, m.ups[s], gp + "ups." + std::to_string(s), cin, c, k, true, true, 1, u);
    int sf = 1;
    for (int j = s + 1; j < nup; ++j) sf *= m.rates[j];
    const bool last = s + 1 == nup;
    const int nk = last ? 1 : 2 * sf;
    if (ist) {
      add_wconv(m, m.nc_conv[s], gp + "noise_convs." + std::to_string(s), m.n_fft + 2, c, nk, false, true);
    } else if (nk >= 16 && nk == 2 * sf && sf <= 32) {
      // stride-S conv over the source = 2-tap conv over S-sample frames (k_har_frames)
      add_wconv(m, m.nc_mm[s], gp + "noise_convs." + std::to_string(s), sf, c, 2, false, true);
      m.nc_mm[s].reframe = sf;
      m.nc_w.push_back(-1);
      m.nc_b.push_back(-1);
    } else {
      m.nc_w.push_back(m.P.add(gp + "noise_convs." + std::to_string(s) + ".weight", (long long)c * nk));
      m.nc_b.push_back(m.P.add(gp + "noise_convs." + std::to_string(s) + ".bias", c));
    }
    add_resblock1(m, m.noise_res[s], gp + "noise_res." + std::to_string(s), c, last ? 11 : 7, d135);
  }
  if (!ist) m.alphas.push_back(m.P.add("generator.alphas.0", m.init_ch));
  for (int s = 0; s < nup; ++s) {
    const int c = m.init_ch >> (s + 1);
    if (!ist) m.alphas.push_back(m.P.add("generator.alphas." + std::to_string(s + 1), c));
    for (int j = 0; j < nrb; ++j)
      add_resblock1(m, m.resblocks[(size_t)s * nrb + j], "generator.resblocks." + std::to_string(s * nrb + j), c,
                    m.rbk[j], m.rbd[j].data());
  }
  const int clast = m.init_ch >> nup;
  add_wconv(m, m.conv_post, "generator.conv_post", clast, ist ? m.n_fft + 2 : 1, 7, true, true);
  if (ist) {
    const int nb = m.n_fft / 2 + 1;
    m.P.add("generator.stft.window", m.n_fft);
    m.stft_fr = m.P.add("generator.stft.weight_forward_real", (long long)nb * m.n_fft);
    m.stft_fi = m.P.add("generator.stft.weight_forward_imag", (long long)nb * m.n_fft);
    m.stft_br = m.P.add("generator.stft.weight_backward_real", (long long)nb * m.n_fft);
    m.stft_bi = m.P.add("generator.stft.weight_backward_imag", (long long)nb * m.n_fft);
  }
  return ST_OK;
}

int build_f0n(Model& m, const int* cfg, int n) {
  if (n != 2 || cfg[0] <= 0 || cfg[0] % 2 || cfg[1] <= 0) return ST_EINVAL;
  m.d_hid = cfg[0];
  m.style_dim = cfg[1];
  const int d = m.d_hid;
  const char* br[2] = {"F0", "N"};
  AdainBlk* blks[2] = {m.f0blk, m.nblk};
  for (int b = 0; b < 2; ++b) {
    const std::string p = br[b];
    add_adainblk(m, blks[b][0], p + ".0", d, d, false);
    add_adainblk(m, blks[b][1], p + ".1", d, d / 2, true);
    add_adainblk(m, blks[b][2], p + ".2", d / 2, d / 2, false);
  }
  add_wconv(m, m.f0_proj, "F0_proj", d / 2, 1, 1, false, true);
  add_wconv(m, m.n_proj, "N_proj", d / 2, 1, 1, false, true);
  return ST_OK;
}

int build_style(Model& m, const int* cfg, int n) {
  if (n != 3 || cfg[0] <= 0 || cfg[1] <= 0 || cfg[2] <= 0) return ST_EINVAL;
  int d = cfg[0];
  m.style_dim = cfg[1];
  add_wconv(m, m.se_conv0, "shared.0", 1, d, 9, false, true);
  for (int i = 0; i < 4; ++i) {
    auto& b = m.se_blk[i];
    const int dout = std::min(d * 2, cfg[2]);
    const std::string p = "shared." + std::to_string(i + 1);
    b.cin = d;
    b.cout = dout;
    b.learned = d != dout;
    add_wconv(m, b.conv1, p + ".conv1", d, d, 9, false, true);
    add_wconv(m, b.conv2, p + ".conv2", d, dout, 9, false, true);
    if (b.learned) add_wconv(m, b.sc, p + ".conv1x1", d, dout, 1, false, false);
    b.dw_w = m.P.add(p + ".downsample_res.conv.weight", (long long)d * 9);
    b.dw_b = m.P.add(p + ".downsample_res.conv.bias", d);
    d = dout;
  }
  add_wconv(m, m.se_last, "shared.6", d, d, 25, false, true);
  m.se_lin_w = m.P.add("unshared.weight", (long long)m.style_dim * d);
  m.se_lin_b = m.P.add("unshared.bias", m.style_dim);
  m.se_dim = d;
  return ST_OK;
}

// MultiPeriodDiscriminator: DiscriminatorP(p) for each period (discriminators.py:132-141); each is
// 5 weight-norm Conv2d (k, 1) stride (3, 1) [the last stride 1] + conv_post (3, 1)
// (discriminators.py:96-106), i.e. 1-d convs along T/p with the same weight memory layout
constexpr int kMpdCh[6] = {1, 32, 128, 512, 1024, 1024};
int build_mpd(Model& m, const int* cfg, int n) {
  if (n < 2 || cfg[0] != n - 1) return ST_EINVAL;
  m.mpd.resize(cfg[0]);  // sized once: add_wconv keeps pointers into it
  for (int i = 0; i < cfg[0]; ++i) {
    if (cfg[1 + i] < 1) return ST_EINVAL;
    auto& d = m.mpd[i];
    d.period = cfg[1 + i];
    const std::string p = "discriminators." + std::to_string(i);
    for (int j = 0; j < 5; ++j)
      add_wconv(m, d.convs[j], p + ".convs." + std::to_string(j), kMpdCh[j], kMpdCh[j + 1], 5, true, true);
    add_wconv(m, d.post, p + ".conv_post", 1024, 1, 3, true, true);
  }
  return ST_OK;
}

// MultiResSpecDiscriminator: SpecDiscriminator(n_fft, hop, win) per resolution (discriminators.py:73-78),
// each 4 weight-norm Conv2d (3, 9) [strides (1,1), (1,2) x 3] + Conv2d (3, 3) + out Conv2d(32, 1, 3)
// (:38-45), cfg = {n, (n_fft, hop, win) x n}
constexpr int kMsdCh = 32;
int g_opt_msdfold = 1;  // STTS_OPT_MSDFOLD, read when an MSD model is created
int build_msd(Model& m, const int* cfg, int n) {
  if (n < 4 || (n - 1) != 3 * cfg[0]) return ST_EINVAL;
  m.msd.resize(cfg[0]);
  for (int i = 0; i < cfg[0]; ++i) {
    auto& d = m.msd[i];
    d.n_fft = cfg[1 + 3 * i];
    d.hop = cfg[2 + 3 * i];
    d.win = cfg[3 + 3 * i];
    if (d.n_fft < 16 || d.n_fft > 2048 || (d.n_fft & (d.n_fft - 1)) || d.hop <= 0 || d.win <= 0 || d.win > d.n_fft)
      return ST_EINVAL;
    const std::string p = "discriminators." + std::to_string(i);
    // a (3, kw) Conv2d runs as a 1-D conv along the bins over 3 C (time-expanded) channels: the
    // reference's [Cout][C][3][kw] weight is exactly the [Cout][3C][kw] Conv1d weight
    for (int j = 0; j < 5; ++j)
      add_wconv(m, d.convs[j], p + ".discriminators." + std::to_string(j), 3 * (j == 0 ? 1 : kMsdCh), kMsdCh,
                j < 4 ? 9 : 3, true, true);
    // the stride (1, 2) layers run folded: stride-1 convs over [W / 2][2 x 96] (N = 32 tiles fill the MFMA
    // columns; the strided tile left 3/4 of them idle)
    if (g_opt_msdfold)
      for (int j = 1; j <= 3; ++j) set_fold(d.convs[j], 2, 4);
    add_wconv(m, d.out, p + ".out", 3 * kMsdCh, 1, 3, true, true);
  }
  return ST_OK;
}

// geometry of SpecDiscriminator over Tn samples: H frames, widths W[0..5] (W[0] = bins; layers 1-3
// halve with kernel 9, pad 4, stride 2)
struct MsdGeom {
  int H, W[6];
};
MsdGeom msd_geom(const Model::DiscS& d, int Tn) {
  MsdGeom g;
  g.H = 1 + Tn / d.hop;
  g.W[0] = g.W[1] = d.n_fft / 2 + 1;
  for (int j = 2; j <= 4; ++j) g.W[j] = (g.W[j - 1] - 1) / 2 + 1;
  g.W[5] = g.W[4];
  return g;
}

long long msd_out_elems(const Model& m, int S, int Tn) {
  long long n = 0;
  for (const auto& d : m.msd) {
    const MsdGeom g = msd_geom(d, Tn);
    for (int j = 1; j <= 5; ++j) n += (long long)S * g.H * g.W[j] * kMsdCh;
    n += (long long)S * g.H * g.W[5];
  }
  return n;
}

// per-layer frame counts of DiscriminatorP(p) over Tn samples: L[0] = ceil(Tn / p), then the 4
// stride-3 convs (k5, pad 2), then the stride-1 conv and conv_post keep L[4]
void mpd_lengths(int Tn, int p, int (&L)[6]) {
  L[0] = (Tn + p - 1) / p;
  for (int j = 0; j < 4; ++j) L[j + 1] = (L[j] + 4 - 5) / 3 + 1;
  L[5] = L[4];
}

long long mpd_out_elems(const Model& m, int B, int Tn) {
  long long n = 0;
  for (const auto& d : m.mpd) {
    int L[6];
    mpd_lengths(Tn, d.period, L);
    for (int j = 0; j < 5; ++j) n += (long long)B * d.period * L[j + 1] * kMpdCh[j + 1];
    n += (long long)B * d.period * L[5];
  }
  return n;
}

void finalize_layout(Model& m) {
  m.Htot = 0;
  for (auto* a : m.adains) {
    a->hoff = m.Htot;
    m.Htot += 2 * a->C;
  }
  for (int dt = 0; dt < ST_NDTYPES; ++dt) {
    const size_t esz = dt == ST_BF16 ? 2 : 4;  // ST_SPLIT: bf16 hi + lo
    size_t off = 0;
    for (auto* c : m.convs) {
      c->off[dt] = off;
      off += rup(st_packed_conv_elems(c->pCin(), c->Cout, c->fold ? c->fK : c->K, c->transposed, c->u) * esz, ALIGN);
    }
    m.conv_bytes[dt] = off;
  }
  // aux fp32 area: AdaIN Wt + bias, folded small convs, pools (dtype independent)
  size_t a = 0;
  m.wt_off = a;
  a += rup((size_t)m.style_dim * m.Htot * 4, ALIGN);
  m.bcat_off = a;
  a += rup((size_t)m.Htot * 4, ALIGN);
  for (auto* s : m.smalls) {
    s->off = a;
    a += rup((size_t)s->rows * s->inner * 4, ALIGN);
  }
  for (auto* p : m.pools) {
    p->pool_off = a;
    a += rup((size_t)p->cin * 3 * 4, ALIGN);
  }
  for (auto* c : m.convs)
    if (c->aux_bias) {
      c->bias_aux = a;
      a += rup((size_t)c->Cout * 4, ALIGN);
    }
  m.aux_bytes = a;
  size_t sc = 0;
  for (auto* c : m.convs) {
    if (c->g >= 0 || c->reframe || c->rs >= 0 || c->src_rows) sc = std::max(sc, (size_t)c->Cin * c->Cout * c->K * 4);
    if (c->fold) sc = std::max(sc, rup((size_t)c->Cin * c->Cout * c->K * 4, ALIGN) + (size_t)c->pCin() * c->Cout * c->fK * 4);
  }
  m.scratch_bytes = rup(sc, ALIGN);
  for (int dt = 0; dt < ST_NDTYPES; ++dt) {
    m.aux_off[dt] = m.conv_bytes[dt];
    m.scratch_off[dt] = m.aux_off[dt] + m.aux_bytes;
    m.total_bytes[dt] = m.scratch_off[dt] + m.scratch_bytes;
  }
}

// ----------------------------------------------------------------------- forward context
struct Buf {
  char* p = nullptr;
  long long bs = 0;  // batch stride (elements)
  int ld = 0, L = 0;
  void* at(int c0, size_t esz) const { return p + (size_t)c0 * esz; }
};

static int g_opt_stats_slots = 0;  // STTS_OPT_STATS_SLOTS (0 = automatic)

struct Ctx {
  Model* m;
  int dtype;  // activation storage (ST_FP32 in the split accuracy mode)
  size_t esz;
  int B;
  hipStream_t s;
  bool dry;
  char* ws;
  size_t off = 0;
  size_t stats_begin = 0, stats_off = 0;
  // small batches: conv statistics spread over `slots` copies so that the persistent grids' fp64
  // atomics do not all land on the same few (utterance, channel) addresses (B = 1: ~200-450 us a
  // launch measured, tools/phase_profile.py with PHASE_B=1), folded after each producing launch
  int slots = 1;
  // small batches: fp32 scratch for the split-K partials of the short-conv engine (pwgemm.hip)
  float* splitk = nullptr;
  long long splitk_elems = 0;
  void alloc_splitk(long long rows_x_cols) {
    if (B > 4) return;
    splitk_elems = 8LL * B * rows_x_cols;  // up to 8 slices
    splitk = reinterpret_cast<float*>(alloc((size_t)splitk_elems * 4));
  }
  float* H = nullptr;
  bool h_ready = false;  // H (every AdaIN layer's style projection) already computed this forward
  const char* packed;
  char* aux;
  int cdtype = 0;  // conv engines / packed weights: the run's dtype (ST_SPLIT in the accuracy mode)

  char* alloc(size_t bytes) {
    char* p = dry ? nullptr : ws + off;
    off += rup(bytes, ALIGN);
    return p;
  }
  Buf frames(int L, int ld) {
    Buf b;
    b.L = L;
    b.ld = ld;
    b.bs = (long long)L * ld;
    b.p = alloc((size_t)B * L * ld * esz);
    return b;
  }
  double* stat(int C) {
    double* p = dry ? nullptr : reinterpret_cast<double*>(ws + stats_off);
    stats_off += rup((size_t)slots * B * C * ST_W * sizeof(double), ALIGN);
    return p;
  }
  const void* wpk(const WConv& c) const { return packed + c.off[cdtype]; }
  const float* aux_f(size_t o) const { return reinterpret_cast<const float*>(aux + o); }
  const float* P(int i) const { return m->P[i]; }
};

#define RUN(expr)                \
  do {                           \
    if (!c.dry) {                \
      int _r = (expr);           \
      if (_r != 0) return _r;    \
    }                            \
  } while (0)

Prologue pro_none() {
  Prologue p;
  memset(&p, 0, sizeof(p));
  return p;
}

Prologue pro_adain(Ctx& c, const WAdaIN& a, const double* stats, int stats_ld, int L, int extra, int alpha,
                   float slope) {
  Prologue p = pro_none();
  p.mode = PRO_AFFINE | extra;
  p.stats = stats;
  p.stats_ld = stats_ld;
  p.inv_n = 1.0 / (double)L;
  p.gamma = c.H ? c.H + a.hoff : nullptr;
  p.gb_ld = c.m->Htot;
  p.gb_C = a.C;
  p.alpha = alpha >= 0 ? c.P(alpha) : nullptr;
  p.slope = slope;
  p.stats_slots = c.slots;  // every stats buffer of the arena has c.slots copies (unused ones zero)
  p.stats_slot_bs = (long long)c.B * stats_ld * ST_W;
  return p;
}

ConvParams conv_base(Ctx& c, const WConv& w, const Buf& x, int c0) {
  ConvParams p;
  memset(&p, 0, sizeof(p));
  p.x = x.at(c0, c.esz);
  p.x_bs = x.bs;
  p.x_ld = x.ld;
  p.Lin = x.L;
  p.Cin = w.pCin();
  p.B = c.B;
  p.KS = w.taps();
  p.dil = 1;
  p.stride = 1;
  p.pad = 0;
  p.N = w.N();
  p.w = c.wpk(w);
  p.nchunks = (w.pCin() + 31) / 32;
  p.bias = w.aux_bias ? c.aux_f(w.bias_aux) : c.P(w.bias);
  p.Cout = w.Cout;
  p.pro = pro_none();
  p.up = 1;
  p.out_scale = 1.0f;
  p.splitk_ws = c.splitk;
  p.splitk_ws_elems = c.splitk_elems;
  return p;
}

void conv_out(ConvParams& p, Ctx& c, const Buf& y, int c0, int Lout) {
  p.y = y.at(c0, c.esz);
  p.y_bs = y.bs;
  p.y_ld = y.ld;
  p.Lout = Lout;
}

// hipEvent pair around one profiled launch (stts_profile_*)
int prof_begin(Ctx& c) {
  while (g_prof.ev.size() < g_prof.used + 2) {
    hipEvent_t e;
    ST_CHECK_HIP(hipEventCreate(&e));
    g_prof.ev.push_back(e);
  }
  ST_CHECK_HIP(hipEventRecord(g_prof.ev[g_prof.used], c.s));
  return 0;
}
int prof_end(Ctx& c, const int (&shape)[8], double fl, double by) {
  ST_CHECK_HIP(hipEventRecord(g_prof.ev[g_prof.used + 1], c.s));
  g_prof.used += 2;
  g_prof.launches++;
  g_prof.flops += fl;
  g_prof.bytes += by;
  Prof::Rec r;
  for (int k = 0; k < 8; ++k) r.shape[k] = shape[k];
  r.flops = fl;
  r.bytes = by;
  g_prof.rec.push_back(r);
  return 0;
}

int conv_run(Ctx& c, ConvParams& p) {
  if (c.dry) return 0;
  const bool prof = g_prof.on;
  if (prof) ST_CHECK(prof_begin(c));
  p.stats_slots = p.stats ? c.slots : 1;
  p.stats_slot_bs = (long long)c.B * p.stats_ld * ST_W;
  int r = st_conv1d(p, c.cdtype, c.s);
  if (r) return r;
  // statistics slots are summed by the consumers' prologues (adain_coeffs): no fold launch
  if (prof) {
    // algorithmic work: a (transposed) conv is 2 * rows * N * Cin * taps flops on its GEMM view;
    // bytes = one read of the input, residual and running sum, one write of the output (none for a
    // statistics-only launch, y == null)
    const double fl = 2.0 * p.B * (double)p.Lq * p.N * p.Cin * p.KS;
    const double outs = (p.y ? 1 : 0) + (p.res ? 1 : 0) + (p.accb ? 1 : 0);
    double elems = (double)p.B * ((double)p.Lin * p.Cin + (double)p.Lout * p.Cout * outs);
    const double by = elems * c.esz + (p.y_f32 ? (double)p.B * p.Lout * p.Cout * (4.0 - c.esz) : 0.0);
    const int flags = (p.res ? 1 : 0) | (p.accb ? 2 : 0) | (st_conv1d_engine(p, c.cdtype) << 4);
    ST_CHECK(prof_end(c, {p.B, p.Lq, p.N, p.Cin, p.KS, p.dil, p.Lout, flags}, fl, by));
  }
  return 0;
}

int resfused_run(Ctx& c, ResFusedParams& p) {
  if (c.dry) return 0;
  const bool prof = g_prof.on;
  if (prof) ST_CHECK(prof_begin(c));
  p.stats_slots = p.stats ? c.slots : 1;
  p.stats_slot_bs = (long long)c.B * p.stats_ld * ST_W;
  ST_CHECK(st_resfused(p, c.s));
  if (prof) {
    // algorithmic work: the statistics pass = conv1 over x (x read once); the fused pass = both convs, x once
    // (window + residual), the running sum, y
    const double fl = (p.stats_only ? 2.0 : 4.0) * p.B * (double)p.L * p.C * p.C * p.K;
    const double by = (double)p.B * p.L * p.C * (p.stats_only ? 1.0 : 2.0 + (p.accb ? 1.0 : 0.0)) * c.esz;
    const int flags = (p.stats_only ? 0 : 1) | (p.accb ? 2 : 0) | (ST_ENGINE_RESFUSED << 4);
    ST_CHECK(prof_end(c, {p.B, p.L, p.C, p.C, p.K, p.dil, p.L, flags}, fl, by));
  }
  return 0;
}

// AdainResBlk1d forward (hifigan.py:390-403).  x frames (ld, L); output into y at channel c0.
int adain_blk(Ctx& c, const AdainBlk& k, const Buf& x, int xc0, const double* st_x, int st_x_ld, const Buf& y,
              int yc0, double* st_y, int st_y_ld, Buf& H1, Buf& SC, Buf& POOL) {
  const int L = x.L, Lr = k.up ? 2 * L : L;
  const float slope = 0.2f;
  // shortcut: conv1x1 at the input rate (nearest x2 commutes with a 1x1 conv)
  if (k.learned) {
    ConvParams p = conv_base(c, k.sc, x, xc0);
    p.Lq = L;
    Buf sc = SC;
    sc.ld = k.cout;
    sc.L = L;
    sc.bs = (long long)L * k.cout;
    conv_out(p, c, sc, 0, L);
    RUN(conv_run(c, p));
  }
  // residual: norm1 -> lrelu -> [pool] -> conv1
  Buf h1 = H1;
  h1.ld = k.cout;
  h1.L = Lr;
  h1.bs = (long long)Lr * k.cout;
  double* st_h1 = c.stat(k.cout);
  {
    ConvParams p;
    if (k.up) {
      Buf pool = POOL;
      pool.ld = rup8(k.cin);
      pool.L = Lr;
      pool.bs = (long long)Lr * pool.ld;
      Prologue pr = pro_adain(c, k.n1, st_x, st_x_ld, L, PRO_LRELU, -1, slope);
      RUN(st_pool_dw(x.at(xc0, c.esz), x.bs, x.ld, c.B, L, k.cin, c.aux_f(k.pool_off), c.P(k.pool_b), pr, pool.p,
                     pool.bs, pool.ld, c.dtype, c.s));
      p = conv_base(c, k.conv1, pool, 0);
    } else {
      p = conv_base(c, k.conv1, x, xc0);
      p.pro = pro_adain(c, k.n1, st_x, st_x_ld, L, PRO_LRELU, -1, slope);
    }
    p.pad = 1;
    p.Lq = Lr;
    conv_out(p, c, h1, 0, Lr);
    p.stats = st_h1;
    p.stats_ld = k.cout;
    RUN(conv_run(c, p));
  }
  // norm2 -> lrelu -> conv2, + shortcut, / sqrt(2)
  {
    ConvParams p = conv_base(c, k.conv2, h1, 0);
    p.pro = pro_adain(c, k.n2, st_h1, k.cout, Lr, PRO_LRELU, -1, slope);
    p.pad = 1;
    p.Lq = Lr;
    conv_out(p, c, y, yc0, Lr);
    if (k.learned) {
      p.res = SC.p;
      p.res_bs = (long long)L * k.cout;
      p.res_ld = k.cout;
    } else {
      p.res = x.at(xc0, c.esz);
      p.res_bs = x.bs;
      p.res_ld = x.ld;
    }
    p.res_shift = k.up ? 1 : 0;
    p.out_scale = (float)(1.0 / sqrt(2.0));
    p.stats = st_y;
    p.stats_ld = st_y_ld;
    RUN(conv_run(c, p));
  }
  return 0;
}

enum ResOut { RO_PLAIN = 0, RO_ACC_FIRST, RO_ACC_MID, RO_ACC_LAST };

// AdaINResBlock1 forward (hifigan.py:65-74).  Input X (stats st_x); temps R, XT; the final
// iteration writes R (RO_PLAIN) or accumulates into ACC (resblock average, hifigan.py:336-342).
int resblock1(Ctx& c, const ResBlock1& rb, const Buf& X, const double* st_x, Buf& R, Buf& XT, int ro, Buf* ACC,
              int nk) {
  const int L = X.L, C = rb.C;
  const Buf* xc = &X;
  const double* st_c = st_x;
  if (st_resfused_eligible(C, rb.K, 1, c.dtype)) {
    // fused iterations (resfused.hip): a statistics pass of conv1, then one launch for
    // conv1 -> AdaIN2 -> Snake2 -> conv2 -> +x.  Outputs ping-pong X -> R -> XT -> R (or ACC):
    // a fused launch reads its input's halos, so it cannot write in place.
    Buf* outs[3] = {&R, &XT, &R};
    for (int d = 0; d < 3; ++d) {
      if (!st_resfused_eligible(C, rb.K, rb.dil[d], c.dtype)) return ST_EINVAL;
      double* st_xt = c.stat(C);
      ResFusedParams f;
      memset(&f, 0, sizeof(f));
      f.x = xc->p;
      f.x_bs = xc->bs;
      f.x_ld = xc->ld;
      f.B = c.B;
      f.L = L;
      f.C = C;
      f.K = rb.K;
      f.dil = rb.dil[d];
      f.w1 = c.wpk(rb.c1[d]);
      f.b1 = c.P(rb.c1[d].bias);
      f.pro1 = pro_adain(c, rb.a1[d], st_c, C, L, PRO_SNAKE, rb.al1[d], 0.f);
      f.stats_only = 1;
      f.stats = st_xt;
      f.stats_ld = C;
      RUN(resfused_run(c, f));
      f.stats_only = 0;
      f.stats = nullptr;
      f.w2 = c.wpk(rb.c2[d]);
      f.b2 = c.P(rb.c2[d].bias);
      f.pro2 = pro_adain(c, rb.a2[d], st_xt, C, L, PRO_SNAKE, rb.al2[d], 0.f);
      const bool final = d == 2;
      const Buf* y = (final && ro != RO_PLAIN) ? ACC : outs[d];
      f.y = y->p;
      f.y_bs = y->bs;
      f.y_ld = y->ld;
      if (final && ro != RO_PLAIN) {
        if (ro != RO_ACC_FIRST) {
          f.accb = ACC->p;
          f.acc_bs = ACC->bs;
          f.acc_ld = ACC->ld;
          if (ro == RO_ACC_LAST) f.acc_div = (float)nk;
        }
      } else if (!final) {
        double* st_r = c.stat(C);
        f.stats = st_r;
        f.stats_ld = C;
        st_c = st_r;
      }
      RUN(resfused_run(c, f));
      xc = outs[d];
    }
    return 0;
  }
  for (int d = 0; d < 3; ++d) {
    double* st_xt = c.stat(C);
    {
      ConvParams p = conv_base(c, rb.c1[d], *xc, 0);
      p.pro = pro_adain(c, rb.a1[d], st_c, C, L, PRO_SNAKE, rb.al1[d], 0.f);
      p.dil = rb.dil[d];
      p.pad = rb.dil[d] * (rb.K - 1) / 2;
      p.Lq = L;
      conv_out(p, c, XT, 0, L);
      p.stats = st_xt;
      p.stats_ld = C;
      RUN(conv_run(c, p));
    }
    {
      ConvParams p = conv_base(c, rb.c2[d], XT, 0);
      p.pro = pro_adain(c, rb.a2[d], st_xt, C, L, PRO_SNAKE, rb.al2[d], 0.f);
      p.pad = (rb.K - 1) / 2;
      p.Lq = L;
      p.res = xc->p;
      p.res_bs = xc->bs;
      p.res_ld = xc->ld;
      const bool final = d == 2;
      if (final && ro != RO_PLAIN) {
        conv_out(p, c, *ACC, 0, L);
        if (ro != RO_ACC_FIRST) {
          p.accb = ACC->p;
          p.acc_bs = ACC->bs;
          p.acc_ld = ACC->ld;
          if (ro == RO_ACC_LAST) p.acc_div = (float)nk;
        }
      } else {
        conv_out(p, c, R, 0, L);
        if (!final) {
          double* st_r = c.stat(C);
          p.stats = st_r;
          p.stats_ld = C;
          st_c = st_r;
        }
      }
      RUN(conv_run(c, p));
    }
    xc = &R;
  }
  return 0;
}

// --------------------------------------------------------------------- decoder forward
struct DecIO {
  const float *asr, *f0, *n, *s, *noise;
  unsigned long long seed;
  long long utt;
  int T;
  float* out;
};

// front-end buffers (hifigan.py:458-472); X0 = decode.3's output [B][2T][512]
struct FrontBufs {
  Buf ENC, CAT[2], H1, SC, POOL, X0;
};

FrontBufs alloc_front(Ctx& c, int T) {
  Model& m = *c.m;
  const int ld_enc = rup8(m.dim_in + 2), ld_cat = rup8(1024 + 2 + 64);
  FrontBufs f;
  f.ENC = c.frames(T, ld_enc);
  f.CAT[0] = c.frames(T, ld_cat);
  f.CAT[1] = c.frames(T, ld_cat);
  f.H1 = c.frames(2 * T, 1024);
  f.SC = c.frames(T, 1024);
  f.POOL = c.frames(2 * T, ld_cat);
  f.X0 = c.frames(2 * T, 512);
  c.H = reinterpret_cast<float*>(c.alloc((size_t)c.B * m.Htot * 4));
  c.alloc_splitk((long long)T * 1024);  // the largest front-end conv output: T x 1024 = 2T x 512
  return f;
}

// the style projections of every AdaIN layer, then the front-end (hifigan.py:458-472 ==
// istftnet.py:704-718 == vocos.py:404-419, eval branch) into f.X0
int run_front(Ctx& c, const DecIO& io, FrontBufs& f) {
  Model& m = *c.m;
  const int B = c.B, T = io.T, n = 2 * T;
  const int ld_enc = rup8(m.dim_in + 2), ld_cat = rup8(1024 + 2 + 64);
  Buf &ENC = f.ENC, *CAT = f.CAT, &H1 = f.H1, &SC = f.SC, &POOL = f.POOL, &X0 = f.X0;
  if (!c.h_ready) RUN(st_linear(io.s, B, m.style_dim, c.aux_f(m.wt_off), c.aux_f(m.bcat_off), m.Htot, c.H, c.s));
  double* S_enc = c.stat(ld_enc);
  RUN(st_ncl_to_frames(io.asr, B, m.dim_in, T, ENC.p, ld_enc, 0, ENC.bs, S_enc, ld_enc, c.dtype, c.s));
  double* S_cat[4];
  for (int k = 0; k < 4; ++k) S_cat[k] = c.stat(ld_cat);
  for (int w = 0; w < 2; ++w) {
    const Small& sm = w == 0 ? m.F0_conv : m.N_conv;
    const float* src = w == 0 ? io.f0 : io.n;
    SmallConvDst d[3];
    d[0] = {ENC.p, ENC.bs, ld_enc, m.dim_in + w, S_enc, ld_enc};
    d[1] = {CAT[0].p, CAT[0].bs, ld_cat, 1024 + 64 + w, S_cat[0], ld_cat};
    d[2] = {CAT[1].p, CAT[1].bs, ld_cat, 1024 + 64 + w, nullptr, 0};
    RUN(st_conv_cin1(src, n, n, B, c.aux_f(sm.off), c.P(sm.bias), 1, 3, 2, 1, T, d, 3, c.dtype, c.s));
  }
  for (int w = 0; w < 2; ++w) {  // asr_res (hifigan.py:438-440, 464) into both concat buffers
    ConvParams p = conv_base(c, m.asr_res, ENC, 0);
    p.Lq = T;
    conv_out(p, c, CAT[w], 1024, T);
    if (w == 0) {
      p.stats = S_cat[0] + 1024 * ST_W;
      p.stats_ld = ld_cat;
    }
    RUN(conv_run(c, p));
    // these statistics are copied slot 0 only into the other concat buffers' stats below: fold
    if (w == 0 && c.slots > 1)
      RUN(st_stats_fold(p.stats, c.B, p.stats_ld, p.Cout, c.slots, (long long)c.B * p.stats_ld * ST_W, c.s));
  }
  if (!c.dry) {  // the constant concat channels share their statistics across the 4 blocks
    for (int k = 1; k < 4; ++k)
      ST_CHECK_HIP(hipMemcpy2DAsync(S_cat[k] + 1024 * ST_W, (size_t)ld_cat * ST_W * 8, S_cat[0] + 1024 * ST_W,
                                    (size_t)ld_cat * ST_W * 8, 66 * ST_W * 8, B, hipMemcpyDeviceToDevice, c.s));
  }
  ST_CHECK(adain_blk(c, m.encode, ENC, 0, S_enc, ld_enc, CAT[0], 0, S_cat[0], ld_cat, H1, SC, POOL));
  ST_CHECK(adain_blk(c, m.decode[0], CAT[0], 0, S_cat[0], ld_cat, CAT[1], 0, S_cat[1], ld_cat, H1, SC, POOL));
  ST_CHECK(adain_blk(c, m.decode[1], CAT[1], 0, S_cat[1], ld_cat, CAT[0], 0, S_cat[2], ld_cat, H1, SC, POOL));
  ST_CHECK(adain_blk(c, m.decode[2], CAT[0], 0, S_cat[2], ld_cat, CAT[1], 0, S_cat[3], ld_cat, H1, SC, POOL));
  ST_CHECK(adain_blk(c, m.decode[3], CAT[1], 0, S_cat[3], ld_cat, X0, 0, nullptr, 0, H1, SC, POOL));
  return 0;
}

int decoder_forward(Ctx& c, const DecIO& io) {
  Model& m = *c.m;
  const int B = c.B, T = io.T;
  const bool ist = m.kind == STTS_KIND_ISTFTNET;
  const int nup = (int)m.rates.size(), nrb = (int)m.rbk.size();
  const size_t esz = c.esz;
  // ---------------- allocations (identical in dry and real runs)
  FrontBufs fb = alloc_front(c, T);
  Buf& X0 = fb.X0;
  const int n = 2 * T;
  int scale = 1;
  for (int r : m.rates) scale *= r;
  if (ist) scale *= m.hop;
  const int L = n * scale;
  float* PH = reinterpret_cast<float*>(c.alloc((size_t)B * 9 * n * 4));
  float* HAR = reinterpret_cast<float*>(c.alloc((size_t)B * L * 4));
  // generator stage geometry
  std::vector<int> Ls(nup), Cs(nup);
  long long smax = 0;
  {
    int Lc = 2 * T;
    for (int s = 0; s < nup; ++s) {
      Lc *= m.rates[s];
      Ls[s] = Lc + ((ist && s == nup - 1) ? 1 : 0);
      Cs[s] = m.init_ch >> (s + 1);
      smax = std::max(smax, (long long)Ls[s] * Cs[s]);
    }
  }
  if (c.cdtype == ST_SPLIT) {  // the fp32 partials of the two-pass C = 64 split resblock convs (ressplit.hip)
    c.splitk_elems = (long long)B * smax;
    c.splitk = reinterpret_cast<float*>(c.alloc((size_t)B * smax * 4));
  }
  Buf G[6];
  for (int i = 0; i < 6; ++i) {
    G[i].p = c.alloc((size_t)B * smax * esz);
    G[i].bs = smax;
  }
  // small batches (STTS_OPT_BRANCHES, default B <= 8): a stage's resblocks 1 .. nrb-1 run beside resblock 0 on side streams, each
  // with its own temporaries and output, averaged afterwards (st_branch_avg) instead of through the running sum:
  // at B = 1 one resblock conv fills 64-512 workgroups, so three side by side fill the chip better.  Not in the
  // split accuracy mode (its two-pass C = 64 convs share the one fp32 partial buffer)
  const bool br = g_opt_branches > 0 && B <= g_opt_branches && nrb > 1 && nrb <= 5 && c.cdtype != ST_SPLIT;
  Buf GB[8];
  // each side-stream resblock also gets its own split-K scratch (the short-conv engine's fp32 partials,
  // st_pw_split): branches that shared c.splitk would write and reduce their partial sums in the same memory
  float* splitk_br[4] = {};
  if (br) {
    for (int i = 0; i < 2 * (nrb - 1); ++i) {
      GB[i].p = c.alloc((size_t)B * smax * esz);
      GB[i].bs = smax;
    }
    if (c.splitk_elems)
      for (int j = 0; j + 1 < nrb; ++j) splitk_br[j] = reinterpret_cast<float*>(c.alloc((size_t)c.splitk_elems * 4));
  }
  Buf HFR;  // S-sample frames of the source for the MFMA noise_convs (largest such stage)
  {
    int rows = 0;
    for (int s = 0; s < nup; ++s)
      if (!ist && m.nc_mm[s].reframe) rows = std::max(rows, Ls[s] + 1);
    if (rows) HFR = c.frames(rows, 32);
    HFR.ld = 32;
  }
  const int F = ist ? L / m.hop + 1 : 0;
  const int ld_h = ist ? rup8(m.n_fft + 2) : 0;
  Buf HARF, POST;
  if (ist) {
    HARF = c.frames(F, ld_h);
    POST = c.frames(F, ld_h);
  }
  // small batches (with the resblock branches): every stage's noise branch (noise_convs -> noise_res, which reads
  // only the harmonic source) runs on a third side stream from the start, beside the front-end and the stages;
  // stage s's ups conv waits for its output (per-stage buffers NSO)
  const bool nbr = (br || (g_opt_nbranch > 0 && B <= g_opt_nbranch && c.cdtype != ST_SPLIT)) && nup <= 8;
  Buf NSO[8], NB[2];
  float* splitk_nb = nullptr;  // the side stream's own split-K scratch (the front-end's short convs use c.splitk)
  if (nbr) {
    for (int s = 0; s < nup; ++s) NSO[s] = c.frames(Ls[s], Cs[s]);
    for (int i = 0; i < 2; ++i) {
      NB[i].p = c.alloc((size_t)B * smax * esz);
      NB[i].bs = smax;
    }
    if (c.splitk_elems) splitk_nb = reinterpret_cast<float*>(c.alloc((size_t)c.splitk_elems * 4));
  }
  c.stats_begin = c.stats_off = c.off;  // stats region follows; its size is known after the dry run
  // ---------------- harmonic source (hifigan.py:323-326 / istftnet.py:544-550)
  RUN(st_sine_phase(io.f0, B, n, scale, PH, c.s));
  RUN(st_sine_source(io.f0, PH, B, n, scale, c.P(m.l_lin_w), c.P(m.l_lin_b), io.noise, io.seed, io.utt, HAR, c.s));
  if (ist) {
    RUN(st_stft(HAR, B, L, m.n_fft, m.hop, c.P(m.stft_fr), c.P(m.stft_fi), HARF.p, ld_h, c.dtype, c.s));
  }
  // noise branch of stage s (hifigan.py:330-331): noise_convs -> NS -> noise_res -> R
  auto noise_branch = [&](int s, Buf NS, Buf R, Buf XT) -> int {
    const int C = Cs[s], Ls_ = Ls[s];
    const bool last = s + 1 == nup;
    double* S_ns = c.stat(C);
    int sf = 1;
    for (int j = s + 1; j < nup; ++j) sf *= m.rates[j];
    if (!ist && m.nc_mm[s].reframe) {  // noise_convs[s] on the MFMA engine over S-sample frames
      const int S = m.nc_mm[s].reframe;
      Buf hf = HFR;
      hf.L = Ls_ + 1;
      hf.bs = (long long)hf.L * 32;
      RUN(st_har_frames(HAR, B, L, S, (S + 1) / 2, Ls_ + 1, 32, hf.p, c.dtype, c.s));
      ConvParams p = conv_base(c, m.nc_mm[s], hf, 0);
      p.Lq = Ls_;
      conv_out(p, c, NS, 0, Ls_);
      p.stats = S_ns;
      p.stats_ld = C;
      RUN(conv_run(c, p));
    } else if (!ist) {
      const int K = last ? 1 : 2 * sf, st = last ? 1 : sf, pd = last ? 0 : (sf + 1) / 2;
      if ((K == 1 || K == 4 || K == 12) && C % 8 == 0 && 256 % (C / 8) == 0) {
        RUN(st_noise_conv(HAR, B, L, c.P(m.nc_w[s]), c.P(m.nc_b[s]), C, K, st, pd, Ls_, NS.p, S_ns, c.dtype, c.s));
      } else {
        SmallConvDst d = {NS.p, NS.bs, C, 0, S_ns, C};
        RUN(st_conv_cin1(HAR, L, L, B, c.P(m.nc_w[s]), c.P(m.nc_b[s]), C, K, st, pd, Ls_, &d, 1, c.dtype, c.s));
      }
    } else {
      Buf hf = HARF;
      ConvParams p = conv_base(c, m.nc_conv[s], hf, 0);
      if (!last) {
        p.stride = sf;
        p.pad = (sf + 1) / 2;
      }
      p.Lq = Ls_;
      conv_out(p, c, NS, 0, Ls_);
      p.stats = S_ns;
      p.stats_ld = C;
      RUN(conv_run(c, p));
    }
    ST_CHECK(resblock1(c, m.noise_res[s], NS, S_ns, R, XT, RO_PLAIN, nullptr, 0));
    return 0;
  };
  auto sview = [&](Buf g, int s) {
    g.ld = Cs[s];
    g.L = Ls[s];
    g.bs = (long long)Ls[s] * Cs[s];
    return g;
  };
  std::unique_lock<std::mutex> branch_lock;
  if ((br || nbr) && !c.dry) branch_lock = std::unique_lock<std::mutex>(m.branch_mu);
  // forked side streams that are not joined back yet: an error return joins them (event on each side stream, the
  // caller's stream waits), so that no side-stream work is left outside a hipGraph capture or still writing the
  // workspace after the call returns
  struct SideJoin {
    hipStream_t main = nullptr;
    hipStream_t s[4] = {};
    hipEvent_t e[4] = {};
    int n = 0;
    void add(hipStream_t st, hipEvent_t ev) {
      s[n] = st;
      e[n] = ev;
      ++n;
    }
    ~SideJoin() {
      for (int i = 0; i < n; ++i) {
        (void)hipEventRecord(e[i], s[i]);
        (void)hipStreamWaitEvent(main, e[i], 0);
      }
    }
  } join_noise, join_br;
  join_noise.main = join_br.main = c.s;
  if (nbr) {
    // the noise branches' AdaIN layers read H (the style projections): computed before the fork
    RUN(st_linear(io.s, B, m.style_dim, c.aux_f(m.wt_off), c.aux_f(m.bcat_off), m.Htot, c.H, c.s));
    c.h_ready = true;
    if (!c.dry) {
      if (!m.side[2]) ST_CHECK_HIP(hipStreamCreateWithFlags(&m.side[2], hipStreamNonBlocking));
      for (int s = 0; s < nup; ++s)
        if (!m.ev_noise[s]) ST_CHECK_HIP(hipEventCreateWithFlags(&m.ev_noise[s], hipEventDisableTiming));
      if (!m.ev_fork2) ST_CHECK_HIP(hipEventCreateWithFlags(&m.ev_fork2, hipEventDisableTiming));
      ST_CHECK_HIP(hipEventRecord(m.ev_fork2, c.s));
      ST_CHECK_HIP(hipStreamWaitEvent(m.side[2], m.ev_fork2, 0));
      join_noise.add(m.side[2], m.ev_noise[nup - 1]);
    }
    const hipStream_t s0 = c.s;
    float* const splitk0 = c.splitk;
    for (int s = 0; s < nup; ++s) {
      if (!c.dry) c.s = m.side[2];
      c.splitk = splitk_nb;
      const int rc = noise_branch(s, sview(NB[0], s), NSO[s], sview(NB[1], s));
      c.splitk = splitk0;
      if (rc == 0 && !c.dry) {
        const int e = (int)hipEventRecord(m.ev_noise[s], c.s);
        c.s = s0;
        ST_CHECK(e);
      }
      c.s = s0;
      ST_CHECK(rc);
    }
  }
  // ---------------- style projections + front-end (hifigan.py:458-472)
  ST_CHECK(run_front(c, io, fb));
  // ---------------- generator stages
  Buf xin = X0;
  int Lcur = 2 * T, Ccur = 512;
  int accsel = 4;
  for (int s = 0; s < nup; ++s) {
    const int u = m.rates[s], C = Cs[s], Ls_ = Ls[s];
    const bool last = s + 1 == nup;
    auto view = [&](Buf g) {
      g.ld = C;
      g.L = Ls_;
      g.bs = (long long)Ls_ * C;
      return g;
    };
    Buf R = view(G[1]), XT = view(G[2]), X = view(G[3]), ACC = view(G[accsel]);
    Buf XS = R;  // x_source: the noise branch's output
    if (nbr) {   // this stage's noise branch ran on the side stream
      XS = NSO[s];
      if (!c.dry) ST_CHECK_HIP(hipStreamWaitEvent(c.s, m.ev_noise[s], 0));
    } else {
      ST_CHECK(noise_branch(s, view(G[0]), R, XT));
    }
    // ups (+ x_source): Snake(alpha_s) / LReLU(0.1) prologue, polyphase ConvTranspose1d
    double* S_x = c.stat(C);
    {
      const WConv& w = m.ups[s];
      ConvParams p = conv_base(c, w, xin, 0);
      p.Cin = Ccur;
      if (!ist) {
        p.pro.mode = PRO_SNAKE;
        p.pro.alpha = c.P(m.alphas[s]);
      } else {
        p.pro.mode = PRO_LRELU;
        p.pro.slope = 0.1f;
      }
      const int taps = w.taps();
      const int padT = ist ? (w.K - u) / 2 : u / 2 + u % 2;
      const int Lout = Lcur * u;
      p.pad = taps - 1;
      p.Lq = (Lout - 1 + padT) / u + 1;
      p.up = u;
      p.opad = padT;
      conv_out(p, c, X, 0, Lout);
      if (ist && last) {
        p.y_row_off = 1;
        p.reflect_front = 1;
      }
      p.res = XS.p;
      p.res_bs = XS.bs;
      p.res_ld = XS.ld;
      p.stats = S_x;
      p.stats_ld = C;
      RUN(conv_run(c, p));
    }
    if (br) {
      // fork: side stream j - 1 runs resblock j after everything queued so far on the caller's stream
      if (!c.dry) {
        for (int j = 0; j + 1 < nrb; ++j) {
          if (!m.side[j]) ST_CHECK_HIP(hipStreamCreateWithFlags(&m.side[j], hipStreamNonBlocking));
          if (!m.ev_join[j]) ST_CHECK_HIP(hipEventCreateWithFlags(&m.ev_join[j], hipEventDisableTiming));
        }
        if (!m.ev_fork) ST_CHECK_HIP(hipEventCreateWithFlags(&m.ev_fork, hipEventDisableTiming));
        ST_CHECK_HIP(hipEventRecord(m.ev_fork, c.s));
        for (int j = 0; j + 1 < nrb; ++j) {
          ST_CHECK_HIP(hipStreamWaitEvent(m.side[j], m.ev_fork, 0));
          join_br.add(m.side[j], m.ev_join[j]);
        }
      }
      ST_CHECK(resblock1(c, m.resblocks[(size_t)s * nrb], X, S_x, R, XT, RO_ACC_FIRST, &ACC, nrb));
      const hipStream_t s0 = c.s;
      float* const splitk0 = c.splitk;
      const void* rs[4];
      for (int j = 1; j < nrb; ++j) {
        Buf Rj = view(GB[2 * (j - 1)]), XTj = view(GB[2 * (j - 1) + 1]);
        if (!c.dry) c.s = m.side[j - 1];
        c.splitk = splitk_br[j - 1];
        const int rc = resblock1(c, m.resblocks[(size_t)s * nrb + j], X, S_x, Rj, XTj, RO_PLAIN, nullptr, 0);
        c.s = s0;
        c.splitk = splitk0;
        ST_CHECK(rc);
        rs[j - 1] = Rj.p;
      }
      // join, then ACC = ((ACC + R_1) + R_2 ...) / nrb
      if (!c.dry) {
        join_br.n = 0;  // joined here
        for (int j = 0; j + 1 < nrb; ++j) {
          ST_CHECK_HIP(hipEventRecord(m.ev_join[j], m.side[j]));
          ST_CHECK_HIP(hipStreamWaitEvent(c.s, m.ev_join[j], 0));
        }
      }
      RUN(st_branch_avg(ACC.p, rs, nrb - 1, (float)nrb, (long long)B * Ls_ * C, c.dtype, c.s));
    } else {
      for (int j = 0; j < nrb; ++j) {
        const int ro = nrb == 1 ? RO_ACC_FIRST : (j == 0 ? RO_ACC_FIRST : (j == nrb - 1 ? RO_ACC_LAST : RO_ACC_MID));
        ST_CHECK(resblock1(c, m.resblocks[(size_t)s * nrb + j], X, S_x, R, XT, ro, &ACC, nrb));
      }
    }
    xin = ACC;
    Lcur = Ls_;
    Ccur = C;
    accsel = accsel == 4 ? 5 : 4;
  }
  join_noise.n = 0;  // every stage waited for its noise branch: the side stream is joined
  // ---------------- output head
  if (!ist) {  // Snake(alpha_last) -> conv_post -> tanh  (hifigan.py:343-345)
    ConvParams p = conv_base(c, m.conv_post, xin, 0);
    p.pro.mode = PRO_SNAKE;
    p.pro.alpha = c.P(m.alphas[nup]);
    p.pad = 3;
    p.Lq = Lcur;
    p.y = io.out;
    p.y_bs = Lcur;
    p.y_ld = 1;
    p.y_f32 = 1;
    p.Lout = Lcur;
    p.epi_tanh = 1;
    RUN(conv_run(c, p));
  } else {  // LReLU(0.01) -> conv_post -> exp/sin -> CustomSTFT.inverse (istftnet.py:569-573)
    ConvParams p = conv_base(c, m.conv_post, xin, 0);
    p.pro.mode = PRO_LRELU;
    p.pro.slope = 0.01f;
    p.pad = 3;
    p.Lq = Lcur;
    conv_out(p, c, POST, 0, Lcur);
    RUN(conv_run(c, p));
    RUN(st_istft(POST.p, B, F, ld_h, m.n_fft, m.hop, c.P(m.stft_br), c.P(m.stft_bi), io.out, L, c.dtype, c.s));
  }
  (void)esz;
  return 0;
}

// --------------------------------------------------------------------- Vocos forward
// Decoder.forward (Modules/vocos.py:392-421, eval): the front-end, then Generator.forward (:157-162):
// per ConvNeXtBlock (:56-69) dwconv (+ InstanceNorm statistics) -> [AdaIN prologue] pwconv1 [GELU
// epilogue] -> pwconv2 with gamma folded [+ residual epilogue]; final LayerNorm; ISTFTHead.out, and
// the exp / clip / cos / sin + irfft + window + overlap-add of ISTFTHead / ISTFT (:271-296, :190-232).
int vocos_forward(Ctx& c, const DecIO& io) {
  Model& m = *c.m;
  const int B = c.B, T = io.T, L = 2 * T, d = m.dim_in;
  FrontBufs fb = alloc_front(c, T);
  Buf XB = c.frames(L, d), D = c.frames(L, d), HI = c.frames(L, m.vc_inter);
  Buf POST = c.frames(L, m.vhead.Cout);
  float* FR = reinterpret_cast<float*>(c.alloc((size_t)B * L * m.n_fft * 4));
  c.stats_begin = c.stats_off = c.off;
  ST_CHECK(run_front(c, io, fb));
  Buf* x = &fb.X0;
  Buf* y = &XB;
  for (const auto& b : m.cnx) {
    double* S_d = c.stat(d);
    RUN(st_dwconv7(x->p, x->bs, x->ld, B, L, d, c.P(b.dw_w), c.P(b.dw_b), D.p, D.bs, D.ld, S_d, d, c.slots,
                   (long long)B * d * ST_W, c.dtype, c.s));
    {
      ConvParams p = conv_base(c, b.pw1, D, 0);
      p.pro = pro_adain(c, b.norm, S_d, d, L, 0, -1, 0.f);
      p.Lq = L;
      conv_out(p, c, HI, 0, L);
      p.epi_gelu = 1;
      RUN(conv_run(c, p));
    }
    {
      ConvParams p = conv_base(c, b.pw2, HI, 0);
      p.Lq = L;
      conv_out(p, c, *y, 0, L);
      p.res = x->p;
      p.res_bs = x->bs;
      p.res_ld = x->ld;
      RUN(conv_run(c, p));
    }
    std::swap(x, y);
  }
  // final LayerNorm (eps 1e-6) into D, the head Linear into POST
  RUN(st_frame_ln(x->p, x->ld, (long long)B * L, d, 1e-6f, c.P(m.ln_w), c.P(m.ln_b), D.p, D.ld, c.dtype, c.s));
  {
    ConvParams p = conv_base(c, m.vhead, D, 0);
    p.Lq = L;
    conv_out(p, c, POST, 0, L);
    RUN(conv_run(c, p));
  }
  RUN(st_istft_head(POST.p, B, L, POST.ld, m.n_fft, m.hop, c.P(m.vwin), FR, io.out, c.dtype, c.s));
  return 0;
}

// --------------------------------------------------------------------- MPD forward
// DiscriminatorP.forward (discriminators.py:108-129) for every period: reflect pad + 1-d -> 2-d
// view (k_period_frames), 5 convs with LeakyReLU(0.1) fused into the epilogue (the activated
// output is the feature map AND the next conv's input), conv_post.  `out` (fp32) receives, per
// period in order, the 6 feature maps as frames [B*p][L_j][C_j] (the reference's [B, C_j, L_j, p]
// tensors permuted; conv_post's map, C = 1, is also the score before flatten).
int mpd_forward(Ctx& c, const float* wave, int Tn, float* out) {
  Model& m = *c.m;
  const int B0 = c.B;
  size_t off = 0;
  for (const auto& d : m.mpd) {
    const int p = d.period;
    int L[6];
    mpd_lengths(Tn, p, L);
    c.B = B0 * p;  // the conv batch: every (utterance, column) sequence
    Buf x = c.frames(L[0], 8);
    RUN(st_period_frames(wave, B0, Tn, p, L[0], x.p, c.dtype, c.s));
    for (int j = 0; j < 5; ++j) {
      Buf y = c.frames(L[j + 1], kMpdCh[j + 1]);
      ConvParams q = conv_base(c, d.convs[j], x, 0);
      q.stride = j < 4 ? 3 : 1;
      q.pad = 2;
      q.Lq = L[j + 1];
      conv_out(q, c, y, 0, L[j + 1]);
      q.epi_lrelu = 1;
      q.epi_slope = 0.1f;  // LRELU_SLOPE (discriminators.py:9)
      RUN(conv_run(c, q));
      RUN(st_frames_to_f32(y.p, c.B, L[j + 1], kMpdCh[j + 1], y.ld, out ? out + off : nullptr, c.dtype, c.s));
      off += (size_t)c.B * L[j + 1] * kMpdCh[j + 1];
      x = y;
    }
    {
      ConvParams q = conv_base(c, d.post, x, 0);
      q.pad = 1;
      q.Lq = L[5];
      q.y = out ? out + off : nullptr;
      q.y_bs = L[5];
      q.y_ld = 1;
      q.y_f32 = 1;
      q.Lout = L[5];
      RUN(conv_run(c, q));
      off += (size_t)c.B * L[5];
    }
    c.B = B0;
  }
  c.stats_begin = c.stats_off = c.off;  // no statistics: the workspace is the buffers above
  return 0;
}

// --------------------------------------------------------------------- MSD forward
// SpecDiscriminator.forward (discriminators.py:47-63) for every resolution over S signals: |STFT| ->
// 4 Conv2d (3, 9) + LeakyReLU(0.1) [the last three with stride (1, 2)] -> Conv2d (3, 3) + LeakyReLU
// -> out Conv2d (3, 3).  Each (3, kw) Conv2d over the (frames, bins) image runs as a 1-D conv along the
// bins of every frame (batch = S * H sequences) over 3 C time-expanded channels (k_time_expand /
// k_stft_mag write x3[h][w][c * 3 + dh] = y[h + dh - 1][w][c]).  `out` (fp32) receives, per resolution,
// the 5 activated feature maps [S][H][W_j][32] and the out map [S][H][W_5] (the reference's
// [S, C, H, W] tensors permuted).
int msd_forward(Ctx& c, const float* wave, int Tn, float* out) {
  Model& m = *c.m;
  const int S = c.B;
  size_t off = 0;
  for (const auto& d : m.msd) {
    const MsdGeom g = msd_geom(d, Tn);
    c.B = S * g.H;  // the conv batch: every (signal, frame) row of bins
    Buf x3 = c.frames(g.W[0], 8);
    if (!c.dry) ST_CHECK_HIP(hipMemsetAsync(x3.p, 0, (size_t)c.B * x3.bs * c.esz, c.s));
    RUN(st_stft_mag_x3(wave, S, Tn, Tn, d.n_fft, d.win, d.hop, x3.p, c.dtype, c.s));
    for (int j = 0; j < 5; ++j) {
      Buf y = c.frames(g.W[j + 1], kMsdCh);
      const WConv& cw = d.convs[j];
      Buf xin = x3;
      if (cw.fold) {  // stride-2 layer, folded: [W_even / 2][2 x 96] rows of the same memory
        xin.L = x3.L / cw.fold;
        xin.ld = x3.ld * cw.fold;
      }
      ConvParams q = conv_base(c, cw, xin, 0);
      q.stride = cw.fold ? 1 : ((j >= 1 && j <= 3) ? 2 : 1);
      q.pad = cw.fold ? cw.fpad : (j < 4 ? 4 : 1);
      q.Lq = g.W[j + 1];
      conv_out(q, c, y, 0, g.W[j + 1]);
      q.epi_lrelu = 1;
      q.epi_slope = 0.1f;  // LRELU_SLOPE (discriminators.py:9)
      RUN(conv_run(c, q));
      RUN(st_frames_to_f32(y.p, c.B, g.W[j + 1], kMsdCh, kMsdCh, out ? out + off : nullptr, c.dtype, c.s));
      off += (size_t)c.B * g.W[j + 1] * kMsdCh;
      // the next layer's input; a folded (stride-2) next layer reads an even number of rows per sequence
      const int fnext = j + 1 < 5 ? d.convs[j + 1].fold : 0;
      const int We = fnext ? (g.W[j + 1] + fnext - 1) / fnext * fnext : g.W[j + 1];
      x3 = c.frames(We, 3 * kMsdCh);
      RUN(st_time_expand(y.p, S, g.H, g.W[j + 1], kMsdCh, x3.p, c.dtype, c.s, We));
    }
    {  // out: Conv2d(32, 1, 3, 1, 1) straight into the fp32 output
      ConvParams q = conv_base(c, d.out, x3, 0);
      q.pad = 1;
      q.Lq = g.W[5];
      q.y = out ? out + off : nullptr;
      q.y_bs = g.W[5];
      q.y_ld = 1;
      q.y_f32 = 1;
      q.Lout = g.W[5];
      RUN(conv_run(c, q));
      off += (size_t)c.B * g.W[5];
    }
    c.B = S;
  }
  c.stats_begin = c.stats_off = c.off;  // no statistics: the workspace is the buffers above
  return 0;
}

// --------------------------------------------------------------------- F0/N forward
int f0n_forward(Ctx& c, const float* x, const float* s, int T, float* F0, float* Nout) {
  Model& m = *c.m;
  const int B = c.B, d = m.d_hid;
  Buf XL = c.frames(T, d);
  Buf Y0 = c.frames(T, d), Y1 = c.frames(2 * T, d / 2), Y2 = c.frames(2 * T, d / 2);
  Buf H1 = c.frames(2 * T, d), SC = c.frames(T, d), POOL = c.frames(2 * T, rup8(d));
  c.H = reinterpret_cast<float*>(c.alloc((size_t)B * m.Htot * 4));
  c.alloc_splitk((long long)T * d);  // the largest conv output of the stacks: T x d = 2T x d/2
  c.stats_begin = c.stats_off = c.off;
  RUN(st_linear(s, B, m.style_dim, c.aux_f(m.wt_off), c.aux_f(m.bcat_off), m.Htot, c.H, c.s));
  double* S0 = c.stat(d);
  RUN(st_frames_convert(x, B, T, d, d, XL.p, d, S0, d, c.dtype, c.s));
  for (int br = 0; br < 2; ++br) {
    AdainBlk* blk = br == 0 ? m.f0blk : m.nblk;
    double* S1 = c.stat(d);
    double* S2 = c.stat(d / 2);
    ST_CHECK(adain_blk(c, blk[0], XL, 0, S0, d, Y0, 0, S1, d, H1, SC, POOL));
    ST_CHECK(adain_blk(c, blk[1], Y0, 0, S1, d, Y1, 0, S2, d / 2, H1, SC, POOL));
    ST_CHECK(adain_blk(c, blk[2], Y1, 0, S2, d / 2, Y2, 0, nullptr, 0, H1, SC, POOL));
    ConvParams p = conv_base(c, br == 0 ? m.f0_proj : m.n_proj, Y2, 0);
    p.Lq = 2 * T;
    p.y = br == 0 ? F0 : Nout;
    p.y_bs = 2 * T;
    p.y_ld = 1;
    p.y_f32 = 1;
    p.Lout = 2 * T;
    RUN(conv_run(c, p));
  }
  return 0;
}

// --------------------------------------------------------------------- style forward
// An image [H][W] is kept zero-padded and row-flattened: row (h+1)*(W+2) + (w+1) holds pixel
// (h, w).  A 3x3 / pad-1 conv is then the 1-D implicit GEMM with 2-level taps
// (row_off = W+2, dil = 1) over output rows q = h*(W+2) + w, written at offset W+3, with the
// two wrap-around columns per image row forced to 0 (they are the next image's padding).
struct Img {
  Buf b;
  int H = 0, W = 0, C = 0;
};

Img img_alloc(Ctx& c, int H, int W, int C) {
  Img im;
  im.H = H;
  im.W = W;
  im.C = C;
  im.b = c.frames((H + 2) * (W + 2), C);
  return im;
}

int conv3x3(Ctx& c, const WConv& w, const Img& x, const Img& y, int pro_lrelu, const Img* res) {
  ConvParams p = conv_base(c, w, x.b, 0);
  p.KS = 9;
  p.kw = 3;
  p.row_off = x.W + 2;
  p.Lq = x.H * (x.W + 2);
  p.zc_period = x.W + 2;
  p.zc_valid = x.W;
  if (pro_lrelu) {
    p.pro.mode = PRO_LRELU;
    p.pro.slope = 0.2f;
  }
  p.y = y.b.p ? y.b.p + (size_t)(x.W + 3) * y.C * c.esz : nullptr;
  p.y_bs = y.b.bs;
  p.y_ld = y.C;
  p.Lout = p.Lq;
  if (res) {
    p.res = res->b.p ? res->b.p + (size_t)(x.W + 3) * res->C * c.esz : nullptr;
    p.res_bs = res->b.bs;
    p.res_ld = res->C;
    p.out_scale = (float)(1.0 / sqrt(2.0));
  }
  return conv_run(c, p);
}

int style_forward(Ctx& c, const float* mel, int T, float* out) {
  Model& m = *c.m;
  const int B = c.B;
  int H = 80, W = T;
  Img M = img_alloc(c, H, W, 8);
  Img A = img_alloc(c, H, W, m.se_conv0.Cout);
  struct BI {
    Img t1, d, scf, scp, y;
  } bi[4];
  {
    int h = H, w = W;
    for (int i = 0; i < 4; ++i) {
      const auto& k = m.se_blk[i];
      const int ho = h / 2, wo = (w + 1) / 2;
      bi[i].t1 = img_alloc(c, h, w, k.cin);
      bi[i].d = img_alloc(c, ho, wo, k.cin);
      if (k.learned) bi[i].scf = img_alloc(c, h, w, k.cout);
      bi[i].scp = img_alloc(c, ho, wo, k.cout);
      bi[i].y = img_alloc(c, ho, wo, k.cout);
      h = ho;
      w = wo;
    }
    if (h < 5 || w < 5) return ST_EINVAL;  // conv 5x5 'valid' needs a 5 x 5 map (T >= 65)
  }
  const Img& X4 = bi[3].y;
  const int Wz = X4.W + 2;
  Buf Z = c.frames(Wz, m.se_dim);
  const size_t style_end = c.off;
  c.stats_begin = c.stats_off = c.off;
  if (!c.dry) ST_CHECK_HIP(hipMemsetAsync(c.ws, 0, style_end, c.s));  // zero image borders
  RUN(st_mel_to_padded(mel, B, H, W, M.b.p, c.dtype, c.s));
  RUN(conv3x3(c, m.se_conv0, M, A, 0, nullptr));
  const Img* x = &A;
  for (int i = 0; i < 4; ++i) {
    const auto& k = m.se_blk[i];
    BI& t = bi[i];
    if (k.learned) {  // shortcut: conv1x1 over every padded row (borders stay 0: no bias)
      ConvParams p = conv_base(c, k.sc, x->b, 0);
      p.Lq = (x->H + 2) * (x->W + 2);
      conv_out(p, c, t.scf.b, 0, p.Lq);
      RUN(conv_run(c, p));
      RUN(st_avgpool_half(t.scf.b.p, B, x->H, x->W, k.cout, t.scp.b.p, c.dtype, c.s));
    } else {
      RUN(st_avgpool_half(x->b.p, B, x->H, x->W, k.cin, t.scp.b.p, c.dtype, c.s));
    }
    RUN(conv3x3(c, k.conv1, *x, t.t1, 1, nullptr));                                     // lrelu -> conv1
    RUN(st_dw_s2(t.t1.b.p, B, x->H, x->W, k.cin, c.P(k.dw_w), c.P(k.dw_b), t.d.b.p, c.dtype, c.s));  // dw s2
    RUN(conv3x3(c, k.conv2, t.d, t.y, 1, &t.scp));                                       // lrelu -> conv2, +sc, /sqrt2
    x = &t.y;
  }
  {  // LeakyReLU -> Conv2d(C, C, 5, 1, 0) over the 5 x W4 map (models.py:137-138)
    ConvParams p = conv_base(c, m.se_last, X4.b, 0);
    p.x = X4.b.p ? X4.b.p + (size_t)(X4.W + 3) * X4.C * c.esz : nullptr;
    p.Lin = (X4.H + 2) * (X4.W + 2) - (X4.W + 3);
    p.KS = 25;
    p.kw = 5;
    p.row_off = X4.W + 2;
    p.Lq = Wz;
    p.zc_period = Wz;
    p.zc_valid = X4.W - 4;
    p.pro.mode = PRO_LRELU;
    p.pro.slope = 0.2f;
    conv_out(p, c, Z, 0, Wz);
    RUN(conv_run(c, p));
  }
  RUN(st_gap_linear(Z.p, B, Wz, X4.W - 4, m.se_dim, c.P(m.se_lin_w), c.P(m.se_lin_b), m.style_dim, out, c.dtype,
                    c.s));
  return 0;
}

// --------------------------------------------------------------------- packing
int pack_model(Model& m, int dt, char* base, hipStream_t s) {
  char* aux = base + m.aux_off[dt];
  float* scratch = reinterpret_cast<float*>(base + m.scratch_off[dt]);
  for (auto* c : m.convs) {
    const float* v = m.P[c->v];
    const float* src = v;
    if (c->g >= 0) {
      const int rows = c->transposed ? c->Cin : c->Cout;
      const long long inner = (long long)c->Cin * c->Cout * c->K / rows;
      ST_CHECK(st_wn_fold(v, m.P[c->g], rows, (int)inner, scratch, s));
      src = scratch;
    } else if (c->reframe) {
      ST_CHECK(st_reframe_w(v, c->Cout, c->reframe, scratch, s));
      src = scratch;
    } else if (c->rs >= 0 || c->src_rows) {
      const int rows = c->src_rows ? c->src_rows : c->Cout;
      ST_CHECK(st_scale_rows(v, c->rs >= 0 ? m.P[c->rs] : nullptr, rows, (long long)c->Cin * c->K, c->Cout, scratch, s));
      src = scratch;
    }
    if (c->aux_bias)
      ST_CHECK(st_scale_rows(m.P[c->bias], c->rs >= 0 ? m.P[c->rs] : nullptr, c->src_rows ? c->src_rows : c->Cout, 1,
                             c->Cout, reinterpret_cast<float*>(aux + c->bias_aux), s));
    if (c->fold) {
      float* fo = scratch + rup((size_t)c->Cin * c->Cout * c->K * 4, ALIGN) / 4;
      ST_CHECK(st_fold_w(src, c->Cout, c->Cin, c->K, c->fold, c->fpad0, c->fK, c->fpad, fo, s));
      src = fo;
    }
    ST_CHECK(st_pack_conv(src, c->pCin(), c->Cout, c->fold ? c->fK : c->K, c->transposed, c->u, base + c->off[dt], dt,
                          s));
  }
  // AdaIN projections: Wt[k][hoff + n] = fc.weight[n][k]; bias concat
  float* Wt = reinterpret_cast<float*>(aux + m.wt_off);
  float* bc = reinterpret_cast<float*>(aux + m.bcat_off);
  for (auto* a : m.adains) {
    ST_CHECK(st_ncl_to_frames(m.P[a->w], 1, 2 * a->C, m.style_dim, Wt, m.Htot, a->hoff, 0, nullptr, 0, ST_FP32, s));
    ST_CHECK_HIP(hipMemcpyAsync(bc + a->hoff, m.P[a->b], (size_t)2 * a->C * 4, hipMemcpyDeviceToDevice, s));
  }
  for (auto* sm : m.smalls)
    ST_CHECK(st_wn_fold(m.P[sm->v], m.P[sm->g], (int)sm->rows, (int)sm->inner,
                        reinterpret_cast<float*>(aux + sm->off), s));
  for (auto* p : m.pools)
    ST_CHECK(st_wn_fold(m.P[p->pool_v], m.P[p->pool_g], p->cin, 3, reinterpret_cast<float*>(aux + p->pool_off), s));
  return 0;
}

int check_params(const Model& m) {
  for (size_t i = 0; i < m.P.ptr.size(); ++i)
    if (!m.P.ptr[i]) return ST_EPARAMS;
  return 0;
}

template <typename F>
int with_ctx(Model* m, int dtype, int B, void* ws, long long ws_bytes, void* stream, F&& body, size_t* need) {
  if (dtype != ST_FP32 && dtype != ST_BF16 && dtype != ST_SPLIT) return ST_EDTYPE;
  const int adt = dtype == ST_BF16 ? ST_BF16 : ST_FP32;  // activation storage
  Ctx c{m, adt, (size_t)(adt == ST_FP32 ? 4 : 2), B, (hipStream_t)stream, true, nullptr};
  c.cdtype = dtype;
  c.slots = g_opt_stats_slots > 0 ? g_opt_stats_slots : (B <= 4 ? 16 : (B <= 16 ? 4 : 1));  // tools/slots_sweep.py
  c.packed = m->packed[dtype];
  c.aux = m->packed[dtype] ? const_cast<char*>(m->packed[dtype]) + m->aux_off[dtype] : nullptr;
  ST_CHECK(body(c));  // dry run: layout
  // the statistics region follows the buffers (stats_off >= off when the body set it); a body
  // without statistics may leave it unset: the buffers alone then size the workspace
  const size_t total = std::max(c.stats_off, c.off);
  if (need) {
    *need = total;
    return 0;
  }
  if (!m->packed[dtype]) return ST_ENOTPACKED;
  if ((long long)total > ws_bytes || !ws) return ST_EWORKSPACE;
  const size_t stats_begin = c.stats_begin;
  Ctx r{m, adt, c.esz, B, (hipStream_t)stream, false, reinterpret_cast<char*>(ws)};
  r.cdtype = dtype;
  r.slots = c.slots;
  r.packed = c.packed;
  r.aux = c.aux;
  if (total > stats_begin) ST_CHECK_HIP(hipMemsetAsync(r.ws + stats_begin, 0, total - stats_begin, r.s));
  return body(r);
}

}  // namespace

// ======================================================================= C-ABI
extern "C" {

int stts_model_create(int kind, const int* cfg, int ncfg, stts_model** out) {
  if (!out || (ncfg > 0 && !cfg)) return ST_EINVAL;
  *out = nullptr;
  Model* m = new Model();
  m->kind = kind;
  int r = ST_EINVAL;
  if (kind == STTS_KIND_HIFIGAN || kind == STTS_KIND_ISTFTNET)
    r = build_decoder(*m, cfg, ncfg);
  else if (kind == STTS_KIND_F0N)
    r = build_f0n(*m, cfg, ncfg);
  else if (kind == STTS_KIND_STYLE)
    r = build_style(*m, cfg, ncfg);
  else if (kind == STTS_KIND_MPD)
    r = build_mpd(*m, cfg, ncfg);
  else if (kind == STTS_KIND_VOCOS)
    r = build_vocos(*m, cfg, ncfg);
  else if (kind == STTS_KIND_MSD)
    r = build_msd(*m, cfg, ncfg);
  if (r != 0) {
    delete m;
    return r;
  }
  finalize_layout(*m);
  *out = m;
  return 0;
}

void stts_model_destroy(stts_model* m) { delete m; }

int stts_param_count(const stts_model* m) { return m ? (int)m->P.names.size() : ST_EINVAL; }

const char* stts_param_name(const stts_model* m, int i) {
  if (!m || i < 0 || i >= (int)m->P.names.size()) return nullptr;
  return m->P.names[i].c_str();
}

long long stts_param_numel(const stts_model* m, int i) {
  if (!m || i < 0 || i >= (int)m->P.names.size()) return ST_EINVAL;
  return m->P.numel[i];
}

int stts_set_param(stts_model* m, int i, const float* p) {
  if (!m || i < 0 || i >= (int)m->P.names.size()) return ST_EINVAL;
  m->P.ptr[i] = p;
  for (auto& pk : m->packed) pk = nullptr;  // weights changed: repack required
  return 0;
}

long long stts_packed_bytes(const stts_model* m, int dtype) {
  if (!m) return ST_EINVAL;
  if (dtype != ST_FP32 && dtype != ST_BF16 && dtype != ST_SPLIT) return ST_EDTYPE;
  return (long long)m->total_bytes[dtype];
}

int stts_pack(stts_model* m, int dtype, void* packed, long long bytes, void* stream) {
  if (!m || !packed) return ST_EINVAL;
  if (dtype != ST_FP32 && dtype != ST_BF16 && dtype != ST_SPLIT) return ST_EDTYPE;
  if (bytes < (long long)m->total_bytes[dtype]) return ST_EWORKSPACE;
  ST_CHECK(check_params(*m));
  ST_CHECK(pack_model(*m, dtype, reinterpret_cast<char*>(packed), (hipStream_t)stream));
  m->packed[dtype] = reinterpret_cast<const char*>(packed);
  return 0;
}

long long stts_workspace_bytes(const stts_model* mc, int dtype, int B, int T) {
  if (!mc || B <= 0 || T <= 0) return ST_EINVAL;
  Model* m = const_cast<Model*>(mc);
  size_t need = 0;
  int r;
  if (m->kind == STTS_KIND_HIFIGAN || m->kind == STTS_KIND_ISTFTNET) {
    DecIO io{};
    io.T = T;
    r = with_ctx(m, dtype, B, nullptr, 0, nullptr, [&](Ctx& c) { return decoder_forward(c, io); }, &need);
  } else if (m->kind == STTS_KIND_F0N) {
    r = with_ctx(m, dtype, B, nullptr, 0, nullptr,
                 [&](Ctx& c) { return f0n_forward(c, nullptr, nullptr, T, nullptr, nullptr); }, &need);
  } else if (m->kind == STTS_KIND_MPD) {
    r = with_ctx(m, dtype, B, nullptr, 0, nullptr, [&](Ctx& c) { return mpd_forward(c, nullptr, T, nullptr); },
                 &need);
  } else if (m->kind == STTS_KIND_MSD) {
    r = with_ctx(m, dtype, B, nullptr, 0, nullptr, [&](Ctx& c) { return msd_forward(c, nullptr, T, nullptr); },
                 &need);
  } else if (m->kind == STTS_KIND_VOCOS) {
    DecIO io{};
    io.T = T;
    r = with_ctx(m, dtype, B, nullptr, 0, nullptr, [&](Ctx& c) { return vocos_forward(c, io); }, &need);
  } else {
    r = with_ctx(m, dtype, B, nullptr, 0, nullptr, [&](Ctx& c) { return style_forward(c, nullptr, T, nullptr); },
                 &need);
  }
  return r ? r : (long long)need;
}

int stts_decoder_fwd(stts_model* m, int dtype, const float* asr, const float* f0, const float* n, const float* s,
                     const float* noise, unsigned long long seed, long long utt_offset, int B, int T, float* out,
                     void* ws, long long ws_bytes, void* stream) {
  if (!m || (m->kind != STTS_KIND_HIFIGAN && m->kind != STTS_KIND_ISTFTNET && m->kind != STTS_KIND_VOCOS))
    return ST_EINVAL;
  if (B <= 0 || T <= 0 || !asr || !f0 || !n || !s || !out) return ST_EINVAL;
  ST_CHECK(check_params(*m));
  DecIO io{asr, f0, n, s, noise, seed, utt_offset, T, out};
  if (m->kind == STTS_KIND_VOCOS)
    return with_ctx(m, dtype, B, ws, ws_bytes, stream, [&](Ctx& c) { return vocos_forward(c, io); }, nullptr);
  return with_ctx(m, dtype, B, ws, ws_bytes, stream, [&](Ctx& c) { return decoder_forward(c, io); }, nullptr);
}

int stts_f0n_fwd(stts_model* m, int dtype, const float* x, const float* s, int B, int T, float* F0, float* N,
                 void* ws, long long ws_bytes, void* stream) {
  if (!m || m->kind != STTS_KIND_F0N) return ST_EINVAL;
  if (B <= 0 || T <= 0 || !x || !s || !F0 || !N) return ST_EINVAL;
  ST_CHECK(check_params(*m));
  return with_ctx(m, dtype, B, ws, ws_bytes, stream, [&](Ctx& c) { return f0n_forward(c, x, s, T, F0, N); },
                  nullptr);
}

int stts_style_fwd(stts_model* m, int dtype, const float* mel, int B, int T, float* out, void* ws, long long ws_bytes,
                   void* stream) {
  if (!m || m->kind != STTS_KIND_STYLE) return ST_EINVAL;
  if (B <= 0 || T <= 0 || !mel || !out) return ST_EINVAL;
  ST_CHECK(check_params(*m));
  return with_ctx(m, dtype, B, ws, ws_bytes, stream, [&](Ctx& c) { return style_forward(c, mel, T, out); }, nullptr);
}

long long stts_mpd_out_elems(const stts_model* m, int B, int T) {
  if (!m || m->kind != STTS_KIND_MPD || B <= 0 || T <= 0) return ST_EINVAL;
  return mpd_out_elems(*m, B, T);
}

int stts_mpd_fwd(stts_model* m, int dtype, const float* wave, int B, int T, float* out, long long out_elems,
                 void* ws, long long ws_bytes, void* stream) {
  if (!m || m->kind != STTS_KIND_MPD) return ST_EINVAL;
  if (B <= 0 || !wave || !out) return ST_EINVAL;
  for (const auto& d : m->mpd)  // the reference's reflect pad needs the pad < T
    if (T < 2 || (T + d.period - 1) / d.period * d.period - T >= T) return ST_EINVAL;
  if (out_elems < mpd_out_elems(*m, B, T)) return ST_EINVAL;
  ST_CHECK(check_params(*m));
  return with_ctx(m, dtype, B, ws, ws_bytes, stream, [&](Ctx& c) { return mpd_forward(c, wave, T, out); }, nullptr);
}

// scratch of stts_mpd_losses / stts_msd_losses: kMpdLossBlocks partial blocks x 4 sums per (discriminator,
// layer) segment (6 per period / resolution)
long long stts_gan_losses_scratch_bytes(const stts_model* m) {
  if (!m) return ST_EINVAL;
  long long segs;
  if (m->kind == STTS_KIND_MPD) segs = 6LL * (long long)m->mpd.size();
  else if (m->kind == STTS_KIND_MSD) segs = 6LL * (long long)m->msd.size();
  else return ST_EINVAL;
  return segs * kMpdLossBlocks * 4 * (long long)sizeof(double);
}

int stts_mpd_losses(const stts_model* m, int B, int T, const float* out, double* scratch,
                    long long scratch_bytes, double* loss, void* stream) {
  if (!m || m->kind != STTS_KIND_MPD || B <= 0 || T <= 0 || !out || !scratch || !loss) return ST_EINVAL;
  MpdLossSegs sg;
  memset(&sg, 0, sizeof(sg));
  long long off = 0;
  for (const auto& d : m->mpd) {
    int L[6];
    mpd_lengths(T, d.period, L);
    for (int j = 0; j < 6; ++j) {
      if (sg.n >= kMpdMaxSegs) return ST_EINVAL;
      const long long half = (long long)B * d.period * L[j < 5 ? j + 1 : 5] * kMpdCh[j < 5 ? j + 1 : 0];
      sg.off[sg.n] = off;
      sg.half[sg.n] = half;
      sg.score[sg.n] = j == 5;
      ++sg.n;
      off += 2 * half;
    }
  }
  if (scratch_bytes < (long long)sg.n * kMpdLossBlocks * 4 * (long long)sizeof(double)) return ST_EWORKSPACE;
  return st_mpd_losses(out, sg, scratch, loss, (hipStream_t)stream);
}

// MultiResolutionSTFTLoss (losses.py:55-94): workspace = the per-resolution partial sums (fixed-order
// reduction) + one resolution's log-mels of both signals (resolutions run one after the other on the stream)
long long stts_mrstft_workspace_bytes(int B, long long L, const int* hops, int n_res, int n_mels) {
  if (B <= 0 || L <= 0 || !hops || n_res <= 0 || n_res > 16 || n_mels <= 0) return ST_EINVAL;
  long long f = 0;
  for (int r = 0; r < n_res; ++r) {
    if (hops[r] <= 0) return ST_EINVAL;
    f = std::max(f, st_stft_frames(L, hops[r]));
  }
  return ((st_sc_part_bytes(n_res) + 255) & ~255LL) + 2LL * B * n_mels * f * 4;
}

int stts_mrstft_loss(const float* x, const float* y, int B, long long L, long long ld, const int* n_ffts,
                     const int* hops, const int* wins, int n_res, int sample_rate, int n_mels, double* loss, void* ws,
                     long long ws_bytes, void* stream) {
  if (!x || !y || !loss || !n_ffts || !hops || !wins || B <= 0 || sample_rate <= 0) return ST_EINVAL;
  const long long need = stts_mrstft_workspace_bytes(B, L, hops, n_res, n_mels);
  if (need < 0) return (int)need;
  if (!ws || ws_bytes < need) return ST_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  double* part = reinterpret_cast<double*>(ws);
  const long long pb = (st_sc_part_bytes(n_res) + 255) & ~255LL;
  float* mx = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + pb);
  for (int r = 0; r < n_res; ++r) {
    const long long F = st_stft_frames(L, hops[r]);
    float* my = mx + (size_t)B * n_mels * F;
    ST_CHECK(st_logmel(x, B, L, ld, n_ffts[r], wins[r], hops[r], n_mels, (float)sample_rate, mx, s));
    ST_CHECK(st_logmel(y, B, L, ld, n_ffts[r], wins[r], hops[r], n_mels, (float)sample_rate, my, s));
    ST_CHECK(st_sc_sums(mx, my, (long long)B * n_mels * F, part + (size_t)r * st_sc_part_bytes(1) / 8, s));
  }
  return st_sc_final(part, n_res, loss, s);
}

long long stts_msd_out_elems(const stts_model* m, int B, int T) {
  if (!m || m->kind != STTS_KIND_MSD || B <= 0 || T <= 0) return ST_EINVAL;
  return msd_out_elems(*m, B, T);
}

int stts_msd_fwd(stts_model* m, int dtype, const float* wave, int B, int T, float* out, long long out_elems,
                 void* ws, long long ws_bytes, void* stream) {
  if (!m || m->kind != STTS_KIND_MSD) return ST_EINVAL;
  if (B <= 0 || !wave || !out) return ST_EINVAL;
  for (const auto& d : m->msd)  // torch.stft's reflect pad needs n_fft / 2 < T
    if (T <= d.n_fft / 2) return ST_EINVAL;
  if (out_elems < msd_out_elems(*m, B, T)) return ST_EINVAL;
  ST_CHECK(check_params(*m));
  return with_ctx(m, dtype, B, ws, ws_bytes, stream, [&](Ctx& c) { return msd_forward(c, wave, T, out); }, nullptr);
}

int stts_msd_losses(const stts_model* m, int B, int T, const float* out, double* scratch,
                    long long scratch_bytes, double* loss, void* stream) {
  if (!m || m->kind != STTS_KIND_MSD || B <= 0 || T <= 0 || !out || !scratch || !loss) return ST_EINVAL;
  MpdLossSegs sg;
  memset(&sg, 0, sizeof(sg));
  long long off = 0;
  for (const auto& d : m->msd) {
    const MsdGeom g = msd_geom(d, T);
    for (int j = 1; j <= 6; ++j) {
      if (sg.n >= kMpdMaxSegs) return ST_EINVAL;
      const long long half = (long long)B * g.H * g.W[j < 6 ? j : 5] * (j < 6 ? kMsdCh : 1);
      sg.off[sg.n] = off;
      sg.half[sg.n] = half;
      sg.score[sg.n] = j == 6;
      ++sg.n;
      off += 2 * half;
    }
  }
  if (scratch_bytes < (long long)sg.n * kMpdLossBlocks * 4 * (long long)sizeof(double)) return ST_EWORKSPACE;
  return st_mpd_losses(out, sg, scratch, loss, (hipStream_t)stream);
}

long long stts_mel_frames(long long L) { return st_mel_frames(L); }

long long stts_mel_workspace_bytes(void) { return st_mel_workspace_bytes(); }

int stts_wave_preprocess(const float* wave, int B, long long L, long long wave_ld, float* mel, void* ws,
                         long long ws_bytes, void* stream) {
  return st_wave_preprocess(wave, B, L, wave_ld, mel, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

int stts_abi_version(void) { return STTS_ABI_VERSION; }

const char* stts_error_string(int code) {
  switch (code) {
    case 0: return "ok";
    case ST_EINVAL: return "invalid argument or shape";
    case ST_EDTYPE: return "unsupported dtype";
    case ST_EPARAMS: return "parameter table incomplete";
    case ST_EWORKSPACE: return "workspace / buffer too small";
    case ST_ENOTPACKED: return "weights not packed for this dtype";
    default: return code > 0 ? hipGetErrorString((hipError_t)code) : "unknown error";
  }
}

int stts_set_option(int key, int value) {
  switch (key) {
    case STTS_OPT_RESCONV: g_opt_resconv = value != 0; return 0;
    case STTS_OPT_GRID_CAP: g_opt_grid_cap = value > 0 ? value : 0; return 0;
    case STTS_OPT_RESFUSED: g_opt_resfused = value != 0; return 0;
    case STTS_OPT_DEBUG: g_opt_debug = value; return 0;
    case STTS_OPT_STATS_SLOTS: g_opt_stats_slots = value > 0 ? value : 0; return 0;
    case STTS_OPT_SMALL_TILES: g_opt_small_tiles = value != 0; return 0;
    case STTS_OPT_BIGCONV: g_opt_bigconv = (value >= 1 && value <= 5) ? value : 2; return 0;
    case STTS_OPT_HEAD: g_opt_head = value ? 1 : 0; return 0;
    case STTS_OPT_SKEW: g_opt_skew = value; return 0;
    case STTS_OPT_FRONT: g_opt_front = (value >= 0 && value <= 2) ? value : 1; return 0;
    case STTS_OPT_PW: g_opt_pw = (value >= 0 && value <= 2) ? value : 1; return 0;
    case STTS_OPT_SPLITK: g_opt_splitk = value ? 1 : 0; return 0;
    case STTS_OPT_EXP: g_opt_exp = value; return 0;
    case STTS_OPT_UPS: g_opt_ups = (value >= 0 && value <= 2) ? value : 1; return 0;
    case STTS_OPT_WGRAD: g_opt_wgw = value ? 1 : 0; return 0;
    case STTS_OPT_PLAINRC: g_opt_plainrc = value ? 1 : 0; return 0;
    case STTS_OPT_MSDFOLD: g_opt_msdfold = value ? 1 : 0; return 0;
    case STTS_OPT_RCPP: g_opt_rcpp = (value >= 0 && value <= 3) ? value : 1; return 0;
    case STTS_OPT_RESSPLIT: g_opt_ressplit = value ? 1 : 0; return 0;
    case STTS_OPT_BIGSPLIT: g_opt_bigsplit = value; return 0;
    case STTS_OPT_BIGLA: g_opt_bigla = value; return 0;
    case STTS_OPT_BIG64: g_opt_big64 = value; return 0;
    case STTS_OPT_BIG3: g_opt_big3 = value; return 0;
    case STTS_OPT_SEGPART: g_opt_segpart = value; return 0;
    case STTS_OPT_RCOCC: g_opt_rcocc = value; return 0;
    case STTS_OPT_BF16F: g_opt_bf16f = value ? 1 : 0; return 0;
    case STTS_OPT_YF32: g_opt_yf32 = value ? 1 : 0; return 0;
    case STTS_OPT_COUT1: g_opt_cout1 = value ? 1 : 0; return 0;
    case STTS_OPT_BRANCHES:
      if (value < 0) return ST_EINVAL;
      g_opt_branches = value;
      return 0;
    case STTS_OPT_NBRANCH:
      if (value < 0) return ST_EINVAL;
      g_opt_nbranch = value;
      return 0;
    default: return ST_EINVAL;
  }
}

int stts_set_debug_buffer(void* buf) {
  g_dbg_stamps = reinterpret_cast<unsigned long long*>(buf);
  return 0;
}

int stts_get_option(int key) {
  switch (key) {
    case STTS_OPT_RESCONV: return g_opt_resconv;
    case STTS_OPT_GRID_CAP: return g_opt_grid_cap;
    case STTS_OPT_RESFUSED: return g_opt_resfused;
    case STTS_OPT_DEBUG: return g_opt_debug;
    case STTS_OPT_STATS_SLOTS: return g_opt_stats_slots;
    case STTS_OPT_SMALL_TILES: return g_opt_small_tiles;
    case STTS_OPT_BIGCONV: return g_opt_bigconv;
    case STTS_OPT_HEAD: return g_opt_head;
    case STTS_OPT_SKEW: return g_opt_skew;
    case STTS_OPT_FRONT: return g_opt_front;
    case STTS_OPT_PW: return g_opt_pw;
    case STTS_OPT_SPLITK: return g_opt_splitk;
    case STTS_OPT_EXP: return g_opt_exp;
    case STTS_OPT_UPS: return g_opt_ups;
    case STTS_OPT_WGRAD: return g_opt_wgw;
    case STTS_OPT_PLAINRC: return g_opt_plainrc;
    case STTS_OPT_MSDFOLD: return g_opt_msdfold;
    case STTS_OPT_RCPP: return g_opt_rcpp;
    case STTS_OPT_RESSPLIT: return g_opt_ressplit;
    case STTS_OPT_BIGSPLIT: return g_opt_bigsplit;
    case STTS_OPT_BIGLA: return g_opt_bigla;
    case STTS_OPT_BIG64: return g_opt_big64;
    case STTS_OPT_BIG3: return g_opt_big3;
    case STTS_OPT_SEGPART: return g_opt_segpart;
    case STTS_OPT_RCOCC: return g_opt_rcocc;
    case STTS_OPT_BF16F: return g_opt_bf16f;
    case STTS_OPT_YF32: return g_opt_yf32;
    case STTS_OPT_COUT1: return g_opt_cout1;
    case STTS_OPT_BRANCHES: return g_opt_branches;
    case STTS_OPT_NBRANCH: return g_opt_nbranch;
    default: return ST_EINVAL;
  }
}

int stts_profile_enable(int on) {
  g_prof.on = on != 0;
  g_prof.used = 0;
  g_prof.launches = 0;
  g_prof.flops = g_prof.bytes = 0;
  g_prof.rec.clear();
  return 0;
}

int stts_profile_launch(long long i, int* shape, double* ms_flops_bytes) {
  if (i < 0 || (size_t)i >= g_prof.rec.size() || 2 * (size_t)i + 1 >= g_prof.used) return ST_EINVAL;
  float ms = 0;
  ST_CHECK_HIP(hipEventSynchronize(g_prof.ev[2 * i + 1]));
  ST_CHECK_HIP(hipEventElapsedTime(&ms, g_prof.ev[2 * i], g_prof.ev[2 * i + 1]));
  const auto& r = g_prof.rec[i];
  if (shape)
    for (int k = 0; k < 8; ++k) shape[k] = r.shape[k];
  if (ms_flops_bytes) {
    ms_flops_bytes[0] = ms;
    ms_flops_bytes[1] = r.flops;
    ms_flops_bytes[2] = r.bytes;
  }
  return 0;
}

int stts_profile_read(double* total_ms, long long* launches, double* alg_flops, double* alg_bytes) {
  double t = 0;
  for (size_t i = 0; i + 1 < g_prof.used; i += 2) {
    float ms = 0;
    ST_CHECK_HIP(hipEventSynchronize(g_prof.ev[i + 1]));
    ST_CHECK_HIP(hipEventElapsedTime(&ms, g_prof.ev[i], g_prof.ev[i + 1]));
    t += ms;
  }
  if (total_ms) *total_ms = t;
  if (launches) *launches = g_prof.launches;
  if (alg_flops) *alg_flops = g_prof.flops;
  if (alg_bytes) *alg_bytes = g_prof.bytes;
  return 0;
}

}  // extern "C"
