// C-ABI implementation: encoder handle, weight packing, workspace layout and the stream-ordered
// forward (ConformerEncoder.forward_for_export, conformer_encoder.py:236-281) built from the
// kernels in gemm.hip / attention.hip / misc.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../include/cfm_encoder.h"
#include "cfm_common.h"
#include "cfm_abi.h"
#include "cfm_kernels.h"
#include "cfm_encoder_impl.h"

using namespace cfm;
namespace cfm {
thread_local KernelClock* g_kclock = nullptr;
}

namespace cfm {
thread_local std::string g_last_error;
}

namespace {

// calc_length (subsampling.py:272-282) in float32 on the host.
int host_calc_length(int len, int repeat) {
  float L = (float)len;
  for (int i = 0; i < repeat; ++i) L = std::floor((L + (2.0f * 1 - 3.0f)) / 2.0f + 1.0f);
  return (int)L;
}

}  // namespace

namespace {

// ---------------------------------------------------------------------------------------------
// parameter table (reference state_dict keys)
// ---------------------------------------------------------------------------------------------
void build_param_list(cfm_encoder* h) {
  auto& P = h->params;
  P.clear();
  const int d = h->d, C = h->C, dff = h->dff, K = h->K, H = h->H;
  P.push_back({"pre_encode.conv.0.weight", (int64_t)C * 9});
  P.push_back({"pre_encode.conv.0.bias", C});
  P.push_back({"pre_encode.conv.2.weight", (int64_t)C * C * 9});
  P.push_back({"pre_encode.conv.2.bias", C});
  P.push_back({"pre_encode.out.weight", (int64_t)d * C * h->F2});
  P.push_back({"pre_encode.out.bias", d});
  for (int l = 0; l < h->L; ++l) {
    const std::string p = "layers." + std::to_string(l) + ".";
    auto ln = [&](const char* n) { P.push_back({p + n + ".weight", d}); P.push_back({p + n + ".bias", d}); };
    auto ff = [&](const char* n) {
      P.push_back({p + n + ".linear1.weight", (int64_t)dff * d}); P.push_back({p + n + ".linear1.bias", dff});
      P.push_back({p + n + ".linear2.weight", (int64_t)d * dff}); P.push_back({p + n + ".linear2.bias", d});
    };
    ln("norm_feed_forward1"); ff("feed_forward1"); ln("norm_conv");
    P.push_back({p + "conv.pointwise_conv1.weight", (int64_t)2 * d * d});
    P.push_back({p + "conv.pointwise_conv1.bias", 2 * d});
    P.push_back({p + "conv.depthwise_conv.weight", (int64_t)d * K});
    P.push_back({p + "conv.depthwise_conv.bias", d});
    P.push_back({p + "conv.batch_norm.weight", d});
    P.push_back({p + "conv.batch_norm.bias", d});
    if (h->cfg.conv_norm_type == 0) {
      P.push_back({p + "conv.batch_norm.running_mean", d});
      P.push_back({p + "conv.batch_norm.running_var", d});
    }
    P.push_back({p + "conv.pointwise_conv2.weight", (int64_t)d * d});
    P.push_back({p + "conv.pointwise_conv2.bias", d});
    ln("norm_self_att");
    for (const char* n : {"linear_q", "linear_k", "linear_v", "linear_out"}) {
      P.push_back({p + "self_attn." + n + ".weight", (int64_t)d * d});
      P.push_back({p + "self_attn." + n + ".bias", d});
    }
    P.push_back({p + "self_attn.linear_pos.weight", (int64_t)d * d});
    P.push_back({p + "self_attn.pos_bias_u", (int64_t)H * h->dk});
    P.push_back({p + "self_attn.pos_bias_v", (int64_t)H * h->dk});
    ln("norm_feed_forward2"); ff("feed_forward2"); ln("norm_out");
  }
  if (h->has_out_proj) {
    P.push_back({"out_proj.weight", (int64_t)h->dout * d});
    P.push_back({"out_proj.bias", h->dout});
  }
}

// ---------------------------------------------------------------------------------------------
// weight packing (host side, once per set_weights)
// ---------------------------------------------------------------------------------------------
struct Packer {
  cfm_encoder* h;
  std::vector<char> buf;
  bool dry = true;
  long off = 0;

  long alloc(long bytes) {
    const long o = round_up(off, 256);
    off = o + bytes;
    if (!dry && (long)buf.size() < off) fail(CFM_ERR_WEIGHTS, "packer overflow");
    return o;
  }
  long f32(const float* src, long n, std::function<float(long)> fn = nullptr) {
    const long o = alloc(n * 4);
    if (!dry) {
      float* dst = (float*)(buf.data() + o);
      for (long i = 0; i < n; ++i) dst[i] = fn ? fn(i) : src[i];
    }
    return o;
  }
  // GEMM bias: N floats zero-padded to the N granule (the GEMM adds bias[n] for every tile column)
  long bias(const float* src, long n) {
    const long np = round_up(n, GEMM_BN);
    return f32(nullptr, np, [=](long i) -> float { return i < n ? src[i] : 0.0f; });
  }
  // W' = val * diag(gamma) packed as mat(), plus the folded-LayerNorm column terms over the packed
  // (rounded) W': c[n] = sum_k W'[n][k], d[n] = sum_k beta[k] val(n, k) + bias(n)  ([Npad] fp32)
  long mat_fold(int N, int K, std::function<float(int, int)> val, const float* gamma, const float* beta,
                std::function<float(int)> bias, long& c_off, long& d_off) {
    const long o = mat(N, K, [&](int n, int k) { return val(n, k) * gamma[k]; });
    const long Npad = round_up(N, GEMM_BN);
    std::vector<float> c(Npad, 0.0f), dd(Npad, 0.0f);
    if (!dry) {
      for (int n = 0; n < N; ++n) {
        double sc = 0.0, sd = 0.0;
        for (int k = 0; k < K; ++k) {
          const float v = val(n, k);
          const float wq = v * gamma[k];
          sc += (h->es == 4) ? (double)wq : (double)host_bf2f(host_f2bf(wq));
          sd += (double)beta[k] * (double)v;
        }
        c[n] = (float)sc;
        dd[n] = (float)(sd + (double)bias(n));
      }
    }
    c_off = f32(nullptr, Npad, [&](long i) { return c[i]; });
    d_off = f32(nullptr, Npad, [&](long i) { return dd[i]; });
    return o;
  }
  // packed [Npad][Kpad] compute-type matrix; val(n, k) for n < N, k < K (others zero)
  long mat(int N, int K, std::function<float(int, int)> val) {
    const long Npad = round_up(N, GEMM_BN), Kp = h->kpad(K);
    const long o = alloc(Npad * Kp * h->es);
    if (!dry) {
      char* base = buf.data() + o;
      std::memset(base, 0, Npad * Kp * h->es);
      for (int n = 0; n < N; ++n)
        for (int k = 0; k < K; ++k) {
          const float v = val(n, k);
          if (v == 0.0f) continue;
          if (h->es == 4) ((float*)base)[(long)n * Kp + k] = v;
          else ((uint16_t*)base)[(long)n * Kp + k] = host_f2bf(v);
        }
    }
    return o;
  }
};

void pack_all(cfm_encoder* h, Packer& pk, const std::map<std::string, const float*>& W) {
  auto get = [&](const std::string& k) -> const float* {
    auto it = W.find(k);
    if (it == W.end()) {
      if (pk.dry) return nullptr;
      fail(CFM_ERR_WEIGHTS, "missing weight: " + k);
    }
    return it->second;
  };
  const int d = h->d, C = h->C, dff = h->dff, K = h->K, H = h->H, dk = h->dk, dkp = h->dkp, F2 = h->F2;
  const float* w;
  // subsampling
  h->conv1_w = pk.f32(get("pre_encode.conv.0.weight"), (long)C * 9);
  h->conv1_b = pk.f32(get("pre_encode.conv.0.bias"), C);
  w = get("pre_encode.conv.2.weight");                          // (C, C, 3, 3) -> [n][tap*C + c]
  h->conv2_w = pk.mat(C, 9 * C, [&](int n, int k) { const int tap = k / C, c = k % C; return w[((long)n * C + c) * 9 + tap]; });
  h->conv2_b = pk.bias(get("pre_encode.conv.2.bias"), C);
  const float* wsub = get("pre_encode.out.weight");             // (d, C*F2) index c*F2+f -> [n][f*C + c]
  h->sub_w = pk.mat(d, F2 * C, [&](int n, int k) { const int f = k / C, c = k % C; return wsub[(long)n * C * F2 + (long)c * F2 + f]; });
  h->sub_b = pk.bias(get("pre_encode.out.bias"), d);
  // all layers' linear_pos stacked: row (l, head, dd) -> W_l[head*dk + dd]
  std::vector<const float*> wpos(h->L);
  for (int l = 0; l < h->L; ++l) wpos[l] = get("layers." + std::to_string(l) + ".self_attn.linear_pos.weight");
  h->pos_w = pk.mat(h->L * H * dkp, d, [&](int n, int k) {
    const int l = n / (H * dkp), r = n % (H * dkp), hh = r / dkp, dd = r % dkp;
    return dd < dk ? wpos[l][(long)(hh * dk + dd) * d + k] : 0.0f;
  });
  h->layers.resize(h->L);
  for (int l = 0; l < h->L; ++l) {
    LayerW& Lw = h->layers[l];
    const std::string p = "layers." + std::to_string(l) + ".";
    auto mat_plain = [&](const std::string& key, int N, int Kk) {
      const float* m = get(key);
      return pk.mat(N, Kk, [=](int n, int k) { return m[(long)n * Kk + k]; });
    };
    Lw.ff1_w1 = mat_plain(p + "feed_forward1.linear1.weight", dff, d);
    Lw.ff1_b1 = pk.bias(get(p + "feed_forward1.linear1.bias"), dff);
    Lw.ff1_w2 = mat_plain(p + "feed_forward1.linear2.weight", d, dff);
    Lw.ff1_b2 = pk.bias(get(p + "feed_forward1.linear2.bias"), d);
    Lw.ff2_w1 = mat_plain(p + "feed_forward2.linear1.weight", dff, d);
    Lw.ff2_b1 = pk.bias(get(p + "feed_forward2.linear1.bias"), dff);
    Lw.ff2_w2 = mat_plain(p + "feed_forward2.linear2.weight", d, dff);
    Lw.ff2_b2 = pk.bias(get(p + "feed_forward2.linear2.bias"), d);
    const float* g_att = get(p + "norm_self_att.weight");
    const float* b_att = get(p + "norm_self_att.bias");
    const float* g_conv = get(p + "norm_conv.weight");
    const float* b_conv = get(p + "norm_conv.bias");
    const float* g_ff2 = get(p + "norm_feed_forward2.weight");
    const float* b_ff2 = get(p + "norm_feed_forward2.bias");
    if (h->ln_fold) {
      const float* w21 = get(p + "feed_forward2.linear1.weight");
      const float* b21 = get(p + "feed_forward2.linear1.bias");
      Lw.ff2_w1f = pk.mat_fold(dff, d, [=](int n, int k) { return w21[(long)n * d + k]; }, g_ff2, b_ff2,
                               [=](int n) { return b21[n]; }, Lw.ff2_lc, Lw.ff2_ld);
    }
    // q | k | v with per-head padding dk -> dkp
    const float* wq[3] = {get(p + "self_attn.linear_q.weight"), get(p + "self_attn.linear_k.weight"),
                          get(p + "self_attn.linear_v.weight")};
    const float* bq[3] = {get(p + "self_attn.linear_q.bias"), get(p + "self_attn.linear_k.bias"),
                          get(p + "self_attn.linear_v.bias")};
    Lw.qkv_w = pk.mat(3 * H * dkp, d, [&](int n, int k) {
      const int part = n / (H * dkp), r = n % (H * dkp), hh = r / dkp, dd = r % dkp;
      return dd < dk ? wq[part][(long)(hh * dk + dd) * d + k] : 0.0f;
    });
    Lw.qkv_b = pk.f32(nullptr, round_up(3 * H * dkp, GEMM_BN), [&](long n) -> float {
      if (n >= 3 * H * dkp) return 0.0f;
      const int part = n / (H * dkp), r = n % (H * dkp), hh = r / dkp, dd = r % dkp;
      return dd < dk ? bq[part][hh * dk + dd] : 0.0f;
    });
    if (h->ln_fold) {
      auto qv = [&](int n, int k) -> float {
        const int part = n / (H * dkp), r = n % (H * dkp), hh = r / dkp, dd = r % dkp;
        return dd < dk ? wq[part][(long)(hh * dk + dd) * d + k] : 0.0f;
      };
      auto qb = [&](int n) -> float {
        const int part = n / (H * dkp), r = n % (H * dkp), hh = r / dkp, dd = r % dkp;
        return dd < dk ? bq[part][hh * dk + dd] : 0.0f;
      };
      Lw.qkv_wf = pk.mat_fold(3 * H * dkp, d, qv, g_att, b_att, qb, Lw.qkv_lc, Lw.qkv_ld);
    }
    Lw.out_w = mat_plain(p + "self_attn.linear_out.weight", d, d);
    Lw.out_b = pk.bias(get(p + "self_attn.linear_out.bias"), d);
    const float* pu = get(p + "self_attn.pos_bias_u");
    const float* pv = get(p + "self_attn.pos_bias_v");
    Lw.uv = pk.f32(nullptr, 2L * H * dkp, [&](long i) -> float {
      const int part = (int)(i / (H * dkp)), r = (int)(i % (H * dkp)), hh = r / dkp, dd = r % dkp;
      return dd < dk ? (part ? pv : pu)[hh * dk + dd] : 0.0f;
    });
    // pointwise_conv1 (2d, d, 1) GLU-packed: 64-col group g = [value 32g.. | gate d+32g..]
    const float* w1 = get(p + "conv.pointwise_conv1.weight");
    const float* b1 = get(p + "conv.pointwise_conv1.bias");
    const int G = (d + 31) / 32;
    auto glu_src = [d](int n) -> int {   // packed column -> source row of pointwise_conv1 (-1: pad)
      const int g = n / 64, j = n % 64, c = g * 32 + (j & 31);
      if (c >= d) return -1;
      return j < 32 ? c : d + c;
    };
    Lw.pw1_w = pk.mat(64 * G, d, [&](int n, int k) { const int s = glu_src(n); return s < 0 ? 0.0f : w1[(long)s * d + k]; });
    Lw.pw1_b = pk.f32(nullptr, round_up(64 * G, GEMM_BN), [&](long n) -> float {
      if (n >= 64 * G) return 0.0f;
      const int s = glu_src((int)n);
      return s < 0 ? 0.0f : b1[s];
    });
    if (h->ln_fold) {
      Lw.pw1_wf = pk.mat_fold(64 * G, d, [&](int n, int k) { const int s = glu_src(n); return s < 0 ? 0.0f : w1[(long)s * d + k]; },
                              g_conv, b_conv, [&](int n) { const int s = glu_src(n); return s < 0 ? 0.0f : b1[s]; },
                              Lw.pw1_lc, Lw.pw1_ld);
    }
    const float* dww = get(p + "conv.depthwise_conv.weight");          // (d, 1, K) -> [K][d]
    Lw.dw_w = pk.f32(nullptr, (long)d * K, [&](long i) -> float { return dww[(i % d) * K + i / d]; });
    Lw.dw_b = pk.f32(get(p + "conv.depthwise_conv.bias"), d);
    Lw.bn_w = pk.f32(get(p + "conv.batch_norm.weight"), d);
    Lw.bn_b = pk.f32(get(p + "conv.batch_norm.bias"), d);
    if (h->cfg.conv_norm_type == 0) {
      Lw.bn_mean = pk.f32(get(p + "conv.batch_norm.running_mean"), d);
      const float* rv = get(p + "conv.batch_norm.running_var");
      Lw.bn_inv = pk.f32(nullptr, d, [&](long i) -> float { return 1.0f / std::sqrt(rv[i] + 1e-5f); });
    } else {
      Lw.bn_mean = Lw.bn_inv = -1;
    }
    Lw.pw2_w = mat_plain(p + "conv.pointwise_conv2.weight", d, d);
    Lw.pw2_b = pk.bias(get(p + "conv.pointwise_conv2.bias"), d);
    const char* lnn[5] = {"norm_feed_forward1", "norm_self_att", "norm_conv", "norm_feed_forward2", "norm_out"};
    for (int i = 0; i < 5; ++i) {
      Lw.ln_w[i] = pk.f32(get(p + lnn[i] + ".weight"), d);
      Lw.ln_b[i] = pk.f32(get(p + lnn[i] + ".bias"), d);
    }
  }
  if (h->has_out_proj) {
    const float* wo = get("out_proj.weight");
    h->outp_w = pk.mat(h->dout, d, [&](int n, int k) { return wo[(long)n * d + k]; });
    h->outp_b = pk.bias(get("out_proj.bias"), h->dout);
  }
}

void build_pe(cfm_encoder* h, int max_len) {
  // RelPositionalEncoding.extend_pe/create_pe (multi_head_attention.py:235-248, 285-294), float32
  const int d = h->d, rows = 2 * max_len - 1;
  std::vector<char> host((size_t)rows * d * h->es);
  const float scale = (float)(-(std::log(10000.0) / d));
  std::vector<float> div(d / 2 + 1);
  for (int i = 0; i < d; i += 2) div[i / 2] = std::exp((float)i * scale);
  for (int r = 0; r < rows; ++r) {
    const float pos = (float)(max_len - 1 - r);
    for (int c = 0; c < d; ++c) {
      const float a = pos * div[c / 2];
      const float v = (c % 2 == 0) ? std::sin(a) : std::cos(a);
      if (h->es == 4) ((float*)host.data())[(long)r * d + c] = v;
      else ((uint16_t*)host.data())[(long)r * d + c] = host_f2bf(v);
    }
  }
  if (h->pe) (void)hipFree(h->pe);
  h->pe = nullptr;
  HIP_OK(hipMalloc(&h->pe, host.size()));
  HIP_OK(hipMemcpy(h->pe, host.data(), host.size(), hipMemcpyHostToDevice));
  h->max_len = max_len;
  if (h->pe_abs) (void)hipFree(h->pe_abs);
  h->pe_abs = nullptr;
  if (h->abs_pos) {
    // PositionalEncoding.extend_pe/create_pe (multi_head_attention.py:235-255): positions 0 .. max_len-1,
    // float32 in every compute mode (it is added to the fp32 residual stream)
    std::vector<float> abs_host((size_t)max_len * d);
    for (int p = 0; p < max_len; ++p)
      for (int c = 0; c < d; ++c) {
        const float a = (float)p * div[c / 2];
        abs_host[(size_t)p * d + c] = (c % 2 == 0) ? std::sin(a) : std::cos(a);
      }
    HIP_OK(hipMalloc(&h->pe_abs, abs_host.size() * 4));
    HIP_OK(hipMemcpy(h->pe_abs, abs_host.data(), abs_host.size() * 4, hipMemcpyHostToDevice));
  }
}

// names of the positional parameters an abs_pos encoder does not have (packed as zeros)
bool is_rel_pos_param(const std::string& key) {
  auto ends = [&](const char* s) {
    const size_t n = std::strlen(s);
    return key.size() >= n && key.compare(key.size() - n, n, s) == 0;
  };
  return ends(".self_attn.linear_pos.weight") || ends(".self_attn.pos_bias_u") || ends(".self_attn.pos_bias_v");
}

void ensure_streams(cfm_encoder* h, int n) {
  while ((int)h->sub_streams.size() < n) {
    hipStream_t st;
    HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    h->sub_streams.push_back(st);
  }
  while ((int)h->sub_events.size() < n + 1) {
    hipEvent_t ev;
    HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    h->sub_events.push_back(ev);
  }
}

// ---------------------------------------------------------------------------------------------
// workspace layout
// ---------------------------------------------------------------------------------------------
struct WsLayout {
  long X1, X2, X, Hn, U, QK, Vt, O, G, S, P, PN, Y, LS, PE, LEN, total;
  int T1, T2, Tp, M, Tpad;
};

// front: the subsampling images X1 / X2 (the full forward); layers-only forwards (T1 = T2 = T',
// no front end) instead hold the caller's positional rows in the compute type (PE).
WsLayout ws_layout_core(const cfm_encoder* h, int B, int T1, int T2, bool front) {
  WsLayout w;
  const long es = h->es;
  w.T1 = T1;
  w.T2 = T2;
  w.Tp = w.T2;
  w.M = B * w.Tp;
  w.Tpad = (int)round_up(std::max(w.Tp, 1), 32);
  long off = 0;
  auto take = [&](long bytes) { const long o = round_up(off, 256); off = o + round_up(bytes, 256) + 256; return o; };
  const long M = w.M;
  // the fused conv.0 + conv.2 kernel needs no X1 image, only its per-pixel input patches
  w.X1 = !front ? -1
       : (h->fuse_conv12 && conv12_supported(h->dtype, h->C)) ? take((long)conv12_patch_bytes(B, w.T1, h->F1, h->C))
                                          : take((long)B * w.T1 * h->F1 * h->C * es);
  w.X2 = front ? take((long)B * w.T2 * h->F2 * h->C * es) : -1;
  w.X = take(M * h->d * 4);
  w.Hn = take(M * h->d * es);
  w.U = take(M * h->dff * es);
  w.QK = take(M * 3 * h->H * h->dkp * es);
  w.Vt = take((long)B * h->H * h->vt_rows * w.Tpad * es);
  w.O = take(M * h->d * es);
  w.G = take(M * h->d * es);
  w.S = take(M * h->d * es);
  w.P = take((long)(2 * w.Tp - 1) * h->L * h->H * h->dkp * es + 64);
  w.PN = h->cfg.conv_norm_type == 1 ? take(M * h->d * 4) : -1;
  w.Y = h->has_out_proj ? take(M * h->dout * 4) : -1;
  w.LS = h->ln_fold ? take(M * ((h->d + LN_GRANULE - 1) / LN_GRANULE) * 8) : -1;   // folded-LayerNorm row partials
  w.PE = front ? -1 : take((long)(2 * w.Tp - 1) * h->d * es);
  w.LEN = front ? -1 : take((long)B * 4);
  w.total = round_up(off, 256);
  return w;
}

WsLayout ws_layout(const cfm_encoder* h, int B, int T) {
  return ws_layout_core(h, B, host_calc_length(T, 1), host_calc_length(T, 2), true);
}

// (q + u) and (q + v) are stored pre-scaled so that exp2(score) == exp(score_ref / sqrt(dk))
float attn_qscale(int dk) { return (float)(1.4426950408889634 / std::sqrt((double)dk)); }

size_t split_workspace(const cfm_encoder* h, int B, int T);

GemmEpi epi_of(int mode, const float* bias, float alpha = 1.0f) {
  GemmEpi e;
  std::memset(&e, 0, sizeof(e));
  e.mode = mode;
  e.bias = bias;
  e.alpha = alpha;
  return e;
}

}  // namespace

// =============================================================================================
// C-ABI
// =============================================================================================
extern "C" {

const char* cfm_last_error(void) { return g_last_error.c_str(); }
int cfm_version(void) { return CFM_ABI_VERSION; }
#ifdef CFM_HALF_F16
int cfm_half_mode(void) { return CFM_COMPUTE_FP16; }
#else
int cfm_half_mode(void) { return CFM_COMPUTE_BF16; }
#endif
int cfm_encoded_length(int len) { return host_calc_length(len, 2); }

cfm_status cfm_encoder_create(const cfm_encoder_cfg* cfg, int device, int compute_mode, cfm_encoder** out) {
  return guarded([&] {
    if (!cfg || !out) fail(CFM_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    if (compute_mode != CFM_COMPUTE_FP32 && compute_mode != CFM_COMPUTE_BF16 && compute_mode != CFM_COMPUTE_FP16)
      fail(CFM_ERR_INVALID_ARG, "compute_mode");
    if (compute_mode != CFM_COMPUTE_FP32 && compute_mode != cfm_half_mode())
      fail(CFM_ERR_UNSUPPORTED, compute_mode == CFM_COMPUTE_FP16 ? "fp16 compute is libcfm_f16.so"
                                                                 : "bf16 compute is libcfm.so");
    if (cfg->subsampling_factor != 4) fail(CFM_ERR_UNSUPPORTED, "only subsampling='striding', factor 4 is implemented");
    if (cfg->d_model <= 0 || cfg->n_heads <= 0 || cfg->d_model % cfg->n_heads) fail(CFM_ERR_INVALID_ARG, "d_model % n_heads");
    if (cfg->d_model % 8) fail(CFM_ERR_UNSUPPORTED, "d_model must be a multiple of 8");
    if (cfg->d_model > 2048) fail(CFM_ERR_UNSUPPORTED, "d_model > 2048");
    if (cfg->conv_kernel_size % 2 == 0 || cfg->conv_kernel_size > 65) fail(CFM_ERR_UNSUPPORTED, "conv_kernel_size");
    if (cfg->feat_in > 262 || cfg->feat_in < 1) fail(CFM_ERR_UNSUPPORTED, "feat_in");
    if (cfg->n_layers < 0) fail(CFM_ERR_INVALID_ARG, "n_layers");
    std::unique_ptr<cfm_encoder> h(new cfm_encoder());
    h->cfg = *cfg;
    h->device = device;
    h->dtype = compute_mode == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16;
    h->es = dtype_size(h->dtype);
    h->bke = GEMM_BK_BYTES / h->es;
    h->d = cfg->d_model;
    h->H = cfg->n_heads;
    h->dk = h->d / h->H;
    h->dkp = (int)round_up(h->dk, 16);
    if (h->dkp > 128) fail(CFM_ERR_UNSUPPORTED, "head dim > 128");
    h->vt_rows = (int)round_up(h->dkp, 32);
    h->dff = h->d * cfg->ff_expansion_factor;
    h->C = cfg->subsampling_conv_channels > 0 ? cfg->subsampling_conv_channels : h->d;
    if (h->C % 8) fail(CFM_ERR_UNSUPPORTED, "subsampling_conv_channels must be a multiple of 8");
    h->F = cfg->feat_in;
    h->F1 = (h->F - 1) / 2 + 1;
    h->F2 = (h->F1 - 1) / 2 + 1;
    h->K = cfg->conv_kernel_size;
    h->L = cfg->n_layers;
    h->has_out_proj = cfg->feat_out > 0 && cfg->feat_out != h->d;
    h->dout = h->has_out_proj ? cfg->feat_out : h->d;
    if (h->dout % 4) fail(CFM_ERR_UNSUPPORTED, "feat_out must be a multiple of 4");
    if (h->dff % 8) fail(CFM_ERR_UNSUPPORTED, "d_ff must be a multiple of 8");
    int prev = 0;
    HIP_OK(hipGetDevice(&prev));
    HIP_OK(hipSetDevice(device));
    build_param_list(h.get());
    HIP_OK(hipMalloc(&h->zero_page, 4096));
    HIP_OK(hipMemset(h->zero_page, 0, 4096));
    build_pe(h.get(), std::max(cfg->pos_emb_max_len, 1));
    if (const char* mb = getenv("CFM_MICROBATCH")) h->microbatches = std::max(1, std::min(8, atoi(mb)));
    h->ln_fold = h->dtype == DT_BF16 && h->d % 4 == 0;
    if (const char* lf = getenv("CFM_LN_FOLD")) h->ln_fold = atoi(lf) != 0 && h->d % 4 == 0;
    if (const char* gd = getenv("CFM_GLU_DW")) h->fuse_glu_dw = atoi(gd) != 0;
    if (const char* cc = getenv("CFM_CONV12")) h->fuse_conv12 = atoi(cc) != 0;
    if (const char* qa = getenv("CFM_QKV_ATTN")) h->fuse_qkv_attn = atoi(qa) != 0;
    ensure_streams(h.get(), 8);
    HIP_OK(hipSetDevice(prev));
    *out = h.release();
  });
}

void cfm_encoder_destroy(cfm_encoder* h) {
  if (!h) return;
  if (h->wbuf) (void)hipFree(h->wbuf);
  if (h->pe) (void)hipFree(h->pe);
  if (h->pe_abs) (void)hipFree(h->pe_abs);
  if (h->zero_page) (void)hipFree(h->zero_page);
  for (auto st : h->sub_streams) (void)hipStreamDestroy(st);
  for (auto ev : h->sub_events) (void)hipEventDestroy(ev);
  delete h;
}

int cfm_encoder_param_count(const cfm_encoder* h) { return h ? (int)h->params.size() : 0; }
const char* cfm_encoder_param_name(const cfm_encoder* h, int i) {
  return (h && i >= 0 && i < (int)h->params.size()) ? h->params[i].first.c_str() : nullptr;
}
int64_t cfm_encoder_param_numel(const cfm_encoder* h, int i) {
  return (h && i >= 0 && i < (int)h->params.size()) ? h->params[i].second : -1;
}

cfm_status cfm_encoder_set_weights(cfm_encoder* h, const cfm_tensor_view* table, int n, void* stream) {
  return guarded([&] {
    if (!h || (!table && n)) fail(CFM_ERR_INVALID_ARG, "null argument");
    int prev = 0;
    HIP_OK(hipGetDevice(&prev));
    HIP_OK(hipSetDevice(h->device));
    if (stream) HIP_OK(hipStreamSynchronize((hipStream_t)stream));
    std::map<std::string, int64_t> expect(h->params.begin(), h->params.end());
    std::map<std::string, std::vector<float>> host;
    std::map<std::string, const float*> W;
    for (int i = 0; i < n; ++i) {
      if (!table[i].name) fail(CFM_ERR_INVALID_ARG, "unnamed tensor");
      const std::string key = table[i].name;
      auto it = expect.find(key);
      if (it == expect.end()) continue;   // e.g. num_batches_tracked
      if (table[i].numel != it->second)
        fail(CFM_ERR_WEIGHTS, "size mismatch for " + key + ": got " + std::to_string(table[i].numel) +
                                  ", expected " + std::to_string(it->second));
      if (table[i].on_device) {
        std::vector<float>& v = host[key];
        v.resize(table[i].numel);
        HIP_OK(hipMemcpy(v.data(), table[i].data, table[i].numel * 4, hipMemcpyDeviceToHost));
        W[key] = v.data();
      } else {
        W[key] = table[i].data;
      }
    }
    // abs_pos: MultiHeadAttention has no linear_pos / pos_bias_u / pos_bias_v - zeros, whatever is passed
    std::vector<float> zeros;
    if (h->abs_pos) {
      int64_t zmax = 0;
      for (auto& kv : expect)
        if (is_rel_pos_param(kv.first)) zmax = std::max(zmax, kv.second);
      zeros.assign((size_t)zmax, 0.0f);
      for (auto& kv : expect)
        if (is_rel_pos_param(kv.first)) W[kv.first] = zeros.data();
    }
    for (auto& kv : expect)
      if (!W.count(kv.first)) fail(CFM_ERR_WEIGHTS, "missing weight: " + kv.first);
    Packer dry{h};
    pack_all(h, dry, W);
    Packer pk{h};
    pk.dry = false;
    pk.buf.assign(round_up(dry.off, 256), 0);
    pack_all(h, pk, W);
    if (h->wbuf && h->wbytes < pk.buf.size()) { HIP_OK(hipFree(h->wbuf)); h->wbuf = nullptr; }
    if (!h->wbuf) { HIP_OK(hipMalloc(&h->wbuf, pk.buf.size())); h->wbytes = pk.buf.size(); }
    HIP_OK(hipMemcpy(h->wbuf, pk.buf.data(), pk.buf.size(), hipMemcpyHostToDevice));
    h->weights_set = true;
    HIP_OK(hipSetDevice(prev));
  });
}

cfm_status cfm_encoder_set_max_audio_length(cfm_encoder* h, int max_audio_length) {
  return guarded([&] {
    if (!h || max_audio_length < 1) fail(CFM_ERR_INVALID_ARG, "bad argument");
    if (max_audio_length <= h->max_len) return;   // extend_pe only grows (multi_head_attention.py:288)
    int prev = 0;
    HIP_OK(hipGetDevice(&prev));
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(hipDeviceSynchronize());
    build_pe(h, max_audio_length);
    HIP_OK(hipSetDevice(prev));
  });
}

int cfm_encoder_max_audio_length(const cfm_encoder* h) { return h ? h->max_len : 0; }

size_t cfm_encoder_workspace_size(const cfm_encoder* h, int B, int T) {
  if (!h || B <= 0 || T <= 0) return 0;
  return std::max(split_workspace(h, B, T), (size_t)ws_layout(h, B, T).total);
}

}  // extern "C"

namespace {

enum Stage { ST_LEN, ST_CONV1, ST_CONV2, ST_SUBOUT, ST_POS, ST_LN, ST_FFN_UP, ST_FFN_DOWN, ST_QKV, ST_ATTN,
             ST_OUTPROJ, ST_PW1, ST_DWCONV, ST_PW2, ST_OUT, ST_QKV_ATTN, ST_COUNT };
const char* kStageNames[ST_COUNT] = {"lengths", "conv1", "conv2_gemm", "subsample_linear", "pos_gemm", "layernorm",
                                     "ffn_up_gemm", "ffn_down_gemm", "qkv_gemm", "rel_attention", "out_proj_gemm",
                                     "pw1_glu_gemm", "dwconv_bn_swish", "pw2_gemm", "output", "qkv_attention"};

// Stage timer (timed entry point only), installed as the thread's KernelClock.
//   packet (default): a start and a stop event in each kernel's own dispatch packet; per-kernel time =
//     the packet's begin -> end (what rocprofv3's kernel trace reports); outputs are the forward's.
//   chain (env CFM_STAGE_CLOCK=chain): one stop event per kernel; per-kernel time = stop(k) - stop(k-1)
//     (includes the dispatch gap and the event's own overhead: ~2.5 us per launch more than packet).
//   burst (env CFM_STAGE_CLOCK=burst): kBurst back-to-back replays between two stream events.
// A stage's time is the sum over its kernels; its launch count the number of kernels per forward.
struct StageTimer final : KernelClock {
  static constexpr int kBurst = 8;
  enum Mode { PACKET, CHAIN, BURST };
  const Mode mode = [] {
    const char* s = getenv("CFM_STAGE_CLOCK");
    if (s && std::string(s) == "burst") return BURST;
    if (s && std::string(s) == "chain") return CHAIN;
    return PACKET;
  }();
  int cur = -1;
  std::vector<hipEvent_t> ev;   // burst / packet: (start, stop) per kernel; chain: marker, then stop per kernel
  std::vector<int> ids;
  hipEvent_t make() {
    hipEvent_t e;
    HIP_OK(hipEventCreate(&e));
    ev.push_back(e);
    return e;
  }
  void mark(int id) { cur = id; }
  int reps() override { return mode == BURST ? kBurst : 1; }
  void begin(hipStream_t st) override {
    ids.push_back(cur);
    if (mode == BURST || (mode == CHAIN && ev.empty())) HIP_OK(hipEventRecord(make(), st));
  }
  hipEvent_t start_event() override { return mode == PACKET ? make() : nullptr; }
  hipEvent_t stop_event() override { return mode == BURST ? nullptr : make(); }
  void end(hipStream_t st) override {
    if (mode == BURST) HIP_OK(hipEventRecord(make(), st));
  }
  void finish(float* ms, int* launches) {
    if (!ev.empty()) HIP_OK(hipEventSynchronize(ev.back()));
    for (size_t i = 0; i < ids.size(); ++i) {
      float t = 0.f;
      if (mode == CHAIN) {
        HIP_OK(hipEventElapsedTime(&t, ev[i], ev[i + 1]));
      } else {
        HIP_OK(hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]));
        if (mode == BURST) t /= kBurst;
      }
      if (ids[i] >= 0 && ids[i] < ST_COUNT) { ms[ids[i]] += t; launches[ids[i]] += 1; }
    }
  }
  ~StageTimer() override { for (auto e : ev) (void)hipEventDestroy(e); }
};
struct ClockGuard {
  explicit ClockGuard(KernelClock* c) { g_kclock = c; }
  ~ClockGuard() { g_kclock = nullptr; }
};
#define TM(id) do { if (tm) tm->mark(id); } while (0)

// linear_pos of every layer at once on pos_emb (2T'-1 rows of d, compute type): by default the
// handle's table window pe[center - T' : center + T' - 1] (batch-independent, multi_head_attention.py:187
// + RelPositionalEncoding.forward :311-313), or a caller's rows (layers-only forward)
void pos_gemm(cfm_encoder* h, int Tp, void* dst, hipStream_t st, const void* pe_rows = nullptr) {
  const long ldp = (long)h->L * h->H * h->dkp;
  GemmEpi e = epi_of(EPI_STORE, nullptr);
  e.C = dst;
  e.ldc = ldp;
  const char* pe_slice = pe_rows ? (const char*)pe_rows : h->pe + (long)(h->max_len - Tp) * h->d * h->es;
  gemm(h->dtype, pe_slice, h->d, 2 * Tp - 1, h->d, h->wbuf + h->pos_w, (int)h->kpad(h->d), (int)ldp, e, h->zero_page,
       st);
}

// The ConformerLayer stack (conformer_modules.py:88-121, 17 x in ConformerEncoder.forward_for_export
// :262-271) on the residual stream X = ws + wl.X (M = B * T' rows of d fp32, the input of layer 0),
// positional projections of every layer at Pbuf; X holds the last layer's norm_out on return (Hn its
// compute-type copy when an out_proj follows).
void run_layer_stack(cfm_encoder* h, char* ws, const WsLayout& wl, int B, const int32_t* lens, const char* Pbuf,
                     hipStream_t st, StageTimer* tm) {
    // CFM_DBG_LAYERS=n (debugging only): run the first n layers (the last of them ends in its norm_out)
    static const int dbg_layers = [] { const char* e = getenv("CFM_DBG_LAYERS"); return e ? atoi(e) : 0; }();
    const int dt = h->dtype, d = h->d, H = h->H, dkp = h->dkp, Tp = wl.Tp, M = wl.M,
              L = dbg_layers > 0 ? std::min(h->L, dbg_layers) : h->L;
    const int es = h->es;
    auto W = [&](long off) { return (const void*)(h->wbuf + off); };
    auto Wf = [&](long off) { return (const float*)(h->wbuf + off); };
    float* X = (float*)(ws + wl.X);
    void* Hn = ws + wl.Hn;
    // LayerNorm fold (bf16 eval): the residual GEMMs ahead of norm_self_att / norm_conv /
    // norm_feed_forward2 also write the new rows in bf16 to Hn and their granule statistics to LS;
    // the next GEMM runs on those rows with gamma folded into its weight (GemmEpi::ln_in)
    const bool fold = h->ln_fold && L > 0;
    const int lnp = (d + LN_GRANULE - 1) / LN_GRANULE;
    float2* lns = fold ? (float2*)(ws + wl.LS) : nullptr;
    auto produce = [&](GemmEpi& r) {
      if (fold) { r.xb = Hn; r.ln_out = lns; r.ln_parts = lnp; }
    };
    auto consume = [&](GemmEpi& e, long lc, long ld) {
      if (!fold) return;
      e.bias = nullptr; e.ln_in = lns; e.ln_parts = lnp; e.ln_width = d; e.ln_c = Wf(lc); e.ln_d = Wf(ld);
    };
    const long ldp = (long)L * H * dkp;
    if (L > 0) {
      TM(ST_LN);
      layernorm(dt, X, M, d, Wf(h->layers[0].ln_w[0]), Wf(h->layers[0].ln_b[0]), nullptr, nullptr, nullptr, Hn, 0, st);
    }

    for (int l = 0; l < L; ++l) {
      const LayerW& Lw = h->layers[l];
      // ---- FFN1 (conformer_modules.py:99-101) ----
      {
        TM(ST_FFN_UP);
        GemmEpi e = epi_of(EPI_SWISH, Wf(Lw.ff1_b1));
        e.C = ws + wl.U; e.ldc = h->dff;
        gemm(dt, Hn, d, M, d, W(Lw.ff1_w1), (int)h->kpad(d), h->dff, e, h->zero_page, st);
        TM(ST_FFN_DOWN);
        GemmEpi r = epi_of(EPI_RESID, Wf(Lw.ff1_b2), 0.5f);
        r.X = X; r.ldx = d;
        produce(r);
        gemm(dt, ws + wl.U, h->dff, M, h->dff, W(Lw.ff1_w2), (int)h->kpad(h->dff), d, r, h->zero_page, st);
      }
      // ---- rel-pos MHSA (conformer_modules.py:103-110) ----
      if (!fold) {
        TM(ST_LN);
        layernorm(dt, X, M, d, Wf(Lw.ln_w[1]), Wf(Lw.ln_b[1]), nullptr, nullptr, nullptr, Hn, 0, st);
      }
      const long qkv_w = fold ? Lw.qkv_wf : Lw.qkv_w;
      if (fold && h->fuse_qkv_attn && qkv_attention_fused_supported(dt, Tp, dkp, d) && (int)h->kpad(d) == d) {
        // the head's q | k | v projection and its attention in one launch (no qkv buffer)
        TM(ST_QKV_ATTN);
        qkv_rel_attention_fused(Hn, d, lns, lnp, W(qkv_w), (int)h->kpad(d), Wf(Lw.qkv_lc), Wf(Lw.qkv_ld), Wf(Lw.uv),
                                attn_qscale(h->dk), Pbuf + (long)l * H * dkp * es, ldp, lens, B, Tp, H, h->dk,
                                h->cfg.att_context_left, h->cfg.att_context_right, ws + wl.O, d, h->zero_page, st);
      } else if (attn_natural_layout(dt, Tp, dkp)) {
        // plain bias GEMM into [q | k | v]; the attention kernel adds u / v, scales and transposes V
        TM(ST_QKV);
        GemmEpi e = epi_of(EPI_STORE, Wf(Lw.qkv_b));
        e.C = ws + wl.QK; e.ldc = 3L * H * dkp;
        consume(e, Lw.qkv_lc, Lw.qkv_ld);
        gemm(dt, Hn, d, M, d, W(qkv_w), (int)h->kpad(d), 3 * H * dkp, e, h->zero_page, st);
        TM(ST_ATTN);
        rel_pos_attention_natural(ws + wl.QK, 3L * H * dkp, Wf(Lw.uv), attn_qscale(h->dk),
                                  Pbuf + (long)l * H * dkp * es, ldp, lens, B, Tp, H, h->dk, dkp,
                                  h->cfg.att_context_left, h->cfg.att_context_right, ws + wl.O, d, st);
      } else {
        TM(ST_QKV);
        GemmEpi e = epi_of(EPI_QKV, Wf(Lw.qkv_b));
        e.C = ws + wl.QK; e.ldc = 3L * H * dkp; e.qk_cols = 2 * H * dkp; e.uv = Wf(Lw.uv);
        e.qscale = attn_qscale(h->dk);
        e.Vt = ws + wl.Vt; e.H = H; e.dkp = dkp; e.vt_rows = h->vt_rows; e.Tpad = wl.Tpad; e.Tp = Tp;
        consume(e, Lw.qkv_lc, Lw.qkv_ld);
        gemm(dt, Hn, d, M, d, W(qkv_w), (int)h->kpad(d), 3 * H * dkp, e, h->zero_page, st);
        TM(ST_ATTN);
        rel_pos_attention(dt, ws + wl.QK, 3L * H * dkp, ws + wl.Vt, h->vt_rows, wl.Tpad,
                          Pbuf + (long)l * H * dkp * es, ldp, lens, B, Tp, H, h->dk,
                          dkp, h->cfg.att_context_left, h->cfg.att_context_right, ws + wl.O, d, st);
      }
      {
        TM(ST_OUTPROJ);
        GemmEpi r = epi_of(EPI_RESID, Wf(Lw.out_b), 1.0f);
        r.X = X; r.ldx = d;
        produce(r);
        gemm(dt, ws + wl.O, d, M, d, W(Lw.out_w), (int)h->kpad(d), d, r, h->zero_page, st);
      }
      // ---- convolution module (conformer_modules.py:112-114, 160-180) ----
      if (!fold) {
        TM(ST_LN);
        layernorm(dt, X, M, d, Wf(Lw.ln_w[2]), Wf(Lw.ln_b[2]), nullptr, nullptr, nullptr, Hn, 0, st);
      }
      if (h->fuse_glu_dw && h->cfg.conv_norm_type == 0 && gemm_glu_dw_supported(dt, Tp, d, h->K)) {
        // pointwise_conv1 + GLU + pad mask + depthwise conv + BatchNorm + Swish in one launch: one
        // 256-row tile per utterance, the GLU output stays in LDS
        TM(ST_PW1);
        GemmEpi e = epi_of(EPI_GLU_DW, Wf(Lw.pw1_b));
        e.C = ws + wl.S; e.ldc = d; e.lens = h->use_pad_mask ? lens : nullptr; e.Tp = Tp;
        e.utt_tp = Tp; e.utt_M = M;
        e.dw_w = Wf(Lw.dw_w); e.dw_b = Wf(Lw.dw_b);
        e.bn_mean = Wf(Lw.bn_mean); e.bn_inv = Wf(Lw.bn_inv); e.bn_w = Wf(Lw.bn_w); e.bn_b = Wf(Lw.bn_b);
        consume(e, Lw.pw1_lc, Lw.pw1_ld);
        gemm_glu_dw(dt, Hn, d, B, Tp, d, W(fold ? Lw.pw1_wf : Lw.pw1_w), (int)h->kpad(d), d, e, h->zero_page, st);
        TM(ST_PW2);
        GemmEpi r = epi_of(EPI_RESID, Wf(Lw.pw2_b), 1.0f);
        r.X = X; r.ldx = d;
        produce(r);
        gemm(dt, ws + wl.S, d, M, d, W(Lw.pw2_w), (int)h->kpad(d), d, r, h->zero_page, st);
      } else {
        TM(ST_PW1);
        GemmEpi e = epi_of(EPI_GLU_MASK, Wf(Lw.pw1_b));
        e.C = ws + wl.G; e.ldc = d; e.lens = h->use_pad_mask ? lens : nullptr; e.Tp = Tp;
        consume(e, Lw.pw1_lc, Lw.pw1_ld);
        gemm(dt, Hn, d, M, d, W(fold ? Lw.pw1_wf : Lw.pw1_w), (int)h->kpad(d), d, e, h->zero_page, st);
        TM(ST_DWCONV);
        if (h->cfg.conv_norm_type == 0) {
          dwconv_norm_swish(dt, ws + wl.G, B, Tp, d, h->K, Wf(Lw.dw_w), Wf(Lw.dw_b), Wf(Lw.bn_mean), Wf(Lw.bn_inv),
                            Wf(Lw.bn_w), Wf(Lw.bn_b), ws + wl.S, nullptr, st);
        } else {
          float* pn = (float*)(ws + wl.PN);
          dwconv_norm_swish(dt, ws + wl.G, B, Tp, d, h->K, Wf(Lw.dw_w), Wf(Lw.dw_b), nullptr, nullptr, nullptr, nullptr,
                            nullptr, pn, st);
          layernorm(dt, pn, M, d, Wf(Lw.bn_w), Wf(Lw.bn_b), nullptr, nullptr, nullptr, ws + wl.S, 1, st);
        }
        TM(ST_PW2);
        GemmEpi r = epi_of(EPI_RESID, Wf(Lw.pw2_b), 1.0f);
        r.X = X; r.ldx = d;
        produce(r);
        gemm(dt, ws + wl.S, d, M, d, W(Lw.pw2_w), (int)h->kpad(d), d, r, h->zero_page, st);
      }
      // ---- FFN2 (conformer_modules.py:116-118) ----
      if (!fold) {
        TM(ST_LN);
        layernorm(dt, X, M, d, Wf(Lw.ln_w[3]), Wf(Lw.ln_b[3]), nullptr, nullptr, nullptr, Hn, 0, st);
      }
      {
        TM(ST_FFN_UP);
        GemmEpi e = epi_of(EPI_SWISH, Wf(Lw.ff2_b1));
        e.C = ws + wl.U; e.ldc = h->dff;
        consume(e, Lw.ff2_lc, Lw.ff2_ld);
        gemm(dt, Hn, d, M, d, W(fold ? Lw.ff2_w1f : Lw.ff2_w1), (int)h->kpad(d), h->dff, e, h->zero_page, st);
        TM(ST_FFN_DOWN);
        GemmEpi r = epi_of(EPI_RESID, Wf(Lw.ff2_b2), 0.5f);
        r.X = X; r.ldx = d;
        gemm(dt, ws + wl.U, h->dff, M, h->dff, W(Lw.ff2_w2), (int)h->kpad(h->dff), d, r, h->zero_page, st);
      }
      // ---- norm_out (conformer_modules.py:120), fused with the next layer's first LayerNorm ----
      const bool next = l + 1 < L;
      const bool want_t = next || h->has_out_proj;
      TM(ST_LN);
      layernorm(dt, X, M, d, Wf(Lw.ln_w[4]), Wf(Lw.ln_b[4]), X, next ? Wf(h->layers[l + 1].ln_w[0]) : nullptr,
                next ? Wf(h->layers[l + 1].ln_b[0]) : nullptr, want_t ? Hn : nullptr, 0, st);
    }

}

void run_forward(cfm_encoder* h, const float* x_bft, const int32_t* len_b, int B, int T, float* y_bdt,
                 int32_t* out_len_b, void* workspace, size_t workspace_bytes, hipStream_t stream, StageTimer* tm,
                 const char* P_ext = nullptr) {
  {
    if (!h || !x_bft || !y_bdt || !out_len_b) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (!h->weights_set) fail(CFM_ERR_WEIGHTS, "weights not set");
    if (B <= 0 || T <= 0) fail(CFM_ERR_INVALID_ARG, "B and T must be positive");
    if (T > h->max_len) fail(CFM_ERR_INVALID_ARG, "T exceeds max_audio_length; call cfm_encoder_set_max_audio_length");
    const WsLayout wl = ws_layout(h, B, T);
    if (!workspace || workspace_bytes < (size_t)wl.total) fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = stream;
    char* ws = (char*)workspace;
    const int dt = h->dtype, d = h->d, H = h->H, dkp = h->dkp, Tp = wl.Tp, M = wl.M, L = h->L;
    const int es = h->es;
    auto W = [&](long off) { return (const void*)(h->wbuf + off); };
    auto Wf = [&](long off) { return (const float*)(h->wbuf + off); };
    float* X = (float*)(ws + wl.X);
    void* Hn = ws + wl.Hn;

    // lengths (subsampling.py:164-171) -> out_len_b, used as the pad mask from here on
    TM(ST_LEN);
    calc_length(len_b, out_len_b, B, T, 2, st);
    const int32_t* lens = out_len_b;

    // ConvSubsampling (subsampling.py:163-176) + xscale (multi_head_attention.py:305-306)
    if (h->fuse_conv12 && conv12_supported(dt, h->C)) {
      // conv.0 + ReLU recomputed inside conv.2's implicit GEMM: no X1 image
      TM(ST_CONV2);
      conv12_fused(x_bft, B, h->F, T, wl.T1, h->F1, wl.T2, h->F2, Wf(h->conv1_w), Wf(h->conv1_b), h->C,
                   W(h->conv2_w), (int)h->kpad(9 * h->C), Wf(h->conv2_b), ws + wl.X2, ws + wl.X1, h->zero_page, st);
    } else {
      TM(ST_CONV1);
      conv1_subsample(dt, x_bft, B, h->F, T, Wf(h->conv1_w), Wf(h->conv1_b), h->C, ws + wl.X1, st);
      TM(ST_CONV2);
      ConvGeom g{ws + wl.X1, wl.T1, h->F1, wl.T2, h->F2, h->C};
      GemmEpi e = epi_of(EPI_RELU, Wf(h->conv2_b));
      e.C = ws + wl.X2;
      e.ldc = h->C;
      gemm_conv(dt, g, B, W(h->conv2_w), (int)h->kpad(9 * h->C), h->C, e, h->zero_page, st);
    }
    {
      TM(ST_SUBOUT);
      const float xs = h->cfg.xscaling ? (float)std::sqrt((double)d) : 1.0f;
      GemmEpi e = epi_of(EPI_SCALE_F32, Wf(h->sub_b), xs);
      e.X = X;
      e.ldx = d;
      gemm(dt, ws + wl.X2, (long)h->F2 * h->C, M, h->F2 * h->C, W(h->sub_w), (int)h->kpad(h->F2 * h->C), d, e,
           h->zero_page, st);
      // abs_pos: PositionalEncoding.forward adds pe[:, :T'] after the xscale (multi_head_attention.py:265-270)
      if (h->abs_pos) add_rows_f32(X, h->pe_abs, B, Tp, d, st);
    }
    const char* Pbuf = P_ext ? P_ext : ws + wl.P;
    if (L > 0 && !P_ext) {
      TM(ST_POS);
      pos_gemm(h, Tp, ws + wl.P, st);
    }
    run_layer_stack(h, ws, wl, B, lens, Pbuf, st, tm);

    const float* fin = X;
    TM(ST_OUT);
    if (h->has_out_proj) {   // out_proj (conformer_encoder.py:277-278)
      if (L == 0) convert_f32(dt, X, Hn, (long)M * d, st);
      GemmEpi e = epi_of(EPI_SCALE_F32, Wf(h->outp_b), 1.0f);
      float* Y = (float*)(ws + wl.Y);
      e.X = Y; e.ldx = h->dout;
      gemm(dt, Hn, d, M, d, W(h->outp_w), (int)h->kpad(d), h->dout, e, h->zero_page, st);
      fin = Y;
    }
    TM(ST_OUT);
    transpose_out(fin, B, Tp, h->dout, y_bdt, st);
    HIP_OK(hipGetLastError());
  }
}

int split_parts(const cfm_encoder* h, int B) { return std::max(1, std::min(h->microbatches, B / 4)); }

// Micro-batch concurrency: utterances are independent (every row of every kernel is computed
// the same way whatever its batch neighbours - tests/test_gpu_encoder.py checks bitwise batch
// invariance), so the batch is split into parts that run on their own streams, forked from and
// joined back into the caller's stream with events (graph-capture safe).  The per-launch latency
// chain of one part's small GEMMs then overlaps another part's work.  The batch-independent
// linear_pos GEMM runs once, before the fork.
size_t split_workspace(const cfm_encoder* h, int B, int T) {
  const int n = split_parts(h, B);
  if (n == 1) return (size_t)ws_layout(h, B, T).total;
  const int bmax = (B + n - 1) / n;
  return (size_t)n * ws_layout(h, bmax, T).total;
}

void run_split(cfm_encoder* h, const float* x_bft, const int32_t* len_b, int B, int T, float* y_bdt,
               int32_t* out_len_b, void* workspace, size_t workspace_bytes, hipStream_t stream) {
  const int n = split_parts(h, B);
  if (n == 1) {
    run_forward(h, x_bft, len_b, B, T, y_bdt, out_len_b, workspace, workspace_bytes, stream, nullptr);
    return;
  }
  if (!h->weights_set) fail(CFM_ERR_WEIGHTS, "weights not set");
  if (T > h->max_len) fail(CFM_ERR_INVALID_ARG, "T exceeds max_audio_length; call cfm_encoder_set_max_audio_length");
  if (!workspace || workspace_bytes < split_workspace(h, B, T)) fail(CFM_ERR_WORKSPACE, "workspace too small");
  ensure_streams(h, n);
  const int bmax = (B + n - 1) / n;
  const WsLayout wl = ws_layout(h, bmax, T);
  char* ws = (char*)workspace;
  const int Tp = wl.Tp;
  const char* P = ws + wl.P;                       // part 0's P region holds the shared projection
  if (h->L > 0) pos_gemm(h, Tp, ws + wl.P, stream);
  HIP_OK(hipEventRecord(h->sub_events[0], stream));
  int b0 = 0;
  for (int i = 0; i < n; ++i) {
    const int bi = B / n + (i < B % n ? 1 : 0);
    hipStream_t si = h->sub_streams[i];
    HIP_OK(hipStreamWaitEvent(si, h->sub_events[0], 0));
    run_forward(h, x_bft + (long)b0 * h->F * T, len_b ? len_b + b0 : nullptr, bi, T,
                y_bdt + (long)b0 * h->dout * Tp, out_len_b + b0, ws + (long)i * wl.total, wl.total, si, nullptr,
                h->L > 0 ? P : nullptr);
    HIP_OK(hipEventRecord(h->sub_events[1 + i], si));
    HIP_OK(hipStreamWaitEvent(stream, h->sub_events[1 + i], 0));
    b0 += bi;
  }
}

}  // namespace

extern "C" {

cfm_status cfm_encoder_forward(cfm_encoder* h, const float* x_bft, const int32_t* len_b, int B, int T, float* y_bdt,
                               int32_t* out_len_b, void* workspace, size_t workspace_bytes, void* stream) {
  return guarded([&] {
    if (!h || !x_bft || !y_bdt || !out_len_b) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (B <= 0 || T <= 0) fail(CFM_ERR_INVALID_ARG, "B and T must be positive");
    run_split(h, x_bft, len_b, B, T, y_bdt, out_len_b, workspace, workspace_bytes, (hipStream_t)stream);
  });
}

size_t cfm_encoder_layers_workspace_size(const cfm_encoder* h, int B, int Tp) {
  if (!h || B <= 0 || Tp <= 0) return 0;
  return (size_t)ws_layout_core(h, B, Tp, Tp, false).total;
}

cfm_status cfm_encoder_layers_forward(cfm_encoder* h, const float* x_btd, const int32_t* len_b, int B, int Tp,
                                      const float* pos_emb, float* y_btd, void* workspace, size_t workspace_bytes,
                                      void* stream) {
  return guarded([&] {
    if (!h || !x_btd || !y_btd) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (!h->weights_set) fail(CFM_ERR_WEIGHTS, "weights not set");
    if (B <= 0 || Tp <= 0) fail(CFM_ERR_INVALID_ARG, "B and T' must be positive");
    if (!pos_emb && Tp > h->max_len) fail(CFM_ERR_INVALID_ARG, "T' exceeds max_audio_length");
    const WsLayout wl = ws_layout_core(h, B, Tp, Tp, false);
    if (!workspace || workspace_bytes < (size_t)wl.total) fail(CFM_ERR_WORKSPACE, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* ws = (char*)workspace;
    const long rows = (long)B * Tp * h->d;
    HIP_OK(hipMemcpyAsync(ws + wl.X, x_btd, rows * 4, hipMemcpyDeviceToDevice, st));
    int32_t* lens = (int32_t*)(ws + wl.LEN);
    calc_length(len_b, lens, B, Tp, 0, st);   // repeat 0: a copy of len_b (T' where NULL)
    if (h->L > 0) {
      const void* pe_rows = nullptr;
      if (pos_emb) {
        convert_f32(h->dtype, pos_emb, ws + wl.PE, (long)(2 * Tp - 1) * h->d, st);
        pe_rows = ws + wl.PE;
      }
      pos_gemm(h, Tp, ws + wl.P, st, pe_rows);
      run_layer_stack(h, ws, wl, B, lens, ws + wl.P, st, nullptr);
    }
    HIP_OK(hipMemcpyAsync(y_btd, ws + wl.X, rows * 4, hipMemcpyDeviceToDevice, st));
    HIP_OK(hipGetLastError());
  });
}

cfm_status cfm_encoder_set_pad_mask(cfm_encoder* h, int on) {
  return guarded([&] {
    if (!h) fail(CFM_ERR_INVALID_ARG, "null handle");
    h->use_pad_mask = on != 0;
  });
}

cfm_status cfm_encoder_set_abs_pos(cfm_encoder* h, int on) {
  return guarded([&] {
    if (!h) fail(CFM_ERR_INVALID_ARG, "null handle");
    if (h->abs_pos == (on != 0)) return;
    int prev = 0;
    HIP_OK(hipGetDevice(&prev));
    HIP_OK(hipSetDevice(h->device));
    HIP_OK(hipDeviceSynchronize());
    h->abs_pos = on != 0;
    build_pe(h, h->max_len);      // (re)builds pe_abs
    h->weights_set = false;       // the positional weights are packed differently: set_weights again
    HIP_OK(hipSetDevice(prev));
  });
}

int cfm_encoder_abs_pos(const cfm_encoder* h) { return h && h->abs_pos ? 1 : 0; }

cfm_status cfm_encoder_set_microbatches(cfm_encoder* h, int n) {
  return guarded([&] {
    if (!h || n < 1 || n > 8) fail(CFM_ERR_INVALID_ARG, "microbatches must be in [1, 8]");
    h->microbatches = n;
  });
}

int cfm_num_stages(void) { return ST_COUNT; }
const char* cfm_stage_name(int i) { return (i >= 0 && i < ST_COUNT) ? kStageNames[i] : nullptr; }

cfm_status cfm_encoder_forward_timed(cfm_encoder* h, const float* x_bft, const int32_t* len_b, int B, int T,
                                     float* y_bdt, int32_t* out_len_b, void* workspace, size_t workspace_bytes,
                                     void* stream, float* stage_ms, int* stage_launches) {
  return guarded([&] {
    if (!stage_ms || !stage_launches) fail(CFM_ERR_INVALID_ARG, "null stage arrays");
    StageTimer tm;
    {
      ClockGuard g(&tm);
      run_forward(h, x_bft, len_b, B, T, y_bdt, out_len_b, workspace, workspace_bytes, (hipStream_t)stream, &tm);
    }
    tm.finish(stage_ms, stage_launches);
  });
}

__global__ void clock_probe_kernel(float* sink) {
  if (sink && threadIdx.x == 0) sink[blockIdx.x] = 0.0f;
}

cfm_status cfm_stage_clock_overhead(void* stream, int n, float* us_per_kernel) {
  return guarded([&] {
    if (n <= 0 || !us_per_kernel) fail(CFM_ERR_INVALID_ARG, "n > 0 and a result pointer");
    StageTimer tm;
    {
      ClockGuard g(&tm);
      for (int i = 0; i < n; ++i) {
        tm.mark(0);
        cfm_launch(clock_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (float*)nullptr);
      }
    }
    std::vector<float> ms(ST_COUNT, 0.0f);
    std::vector<int> cnt(ST_COUNT, 0);
    tm.finish(ms.data(), cnt.data());
    *us_per_kernel = cnt[0] ? 1e3f * ms[0] / (float)cnt[0] : 0.0f;
  });
}

// ---- kernel-level entry points -------------------------------------------------------------

cfm_status cfm_op_layernorm(int dtype, const float* x, int rows, int d, const float* w, const float* b, float* y_f32,
                            void* y_t, void* stream) {
  return guarded([&] {
    if (d % 4 || d > 2048) fail(CFM_ERR_UNSUPPORTED, "d must be a multiple of 4 and <= 2048");
    layernorm(dtype == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16, x, rows, d, w, b, y_f32, nullptr, nullptr, y_t, 0,
              (hipStream_t)stream);
    HIP_OK(hipGetLastError());
  });
}

// The packed operand of cfm_op_linear: [Np][Kp] compute type | fp32 bias [Np] | a 4 KiB zero page.
static size_t linear_pack_bytes(int dt, int N, int K, long* Kp_out = nullptr, long* Np_out = nullptr) {
  const int es = dtype_size(dt);
  const long Kp = round_up(K, GEMM_BK_BYTES / es), Np = round_up(N, GEMM_BN);
  if (Kp_out) *Kp_out = Kp;
  if (Np_out) *Np_out = Np;
  return (size_t)(Np * Kp * es + round_up(Np * 4, 256) + 4096);
}

// w (N, K) fp32 + bias -> pack_ws, on the device and stream-ordered (no host round trip, no sync)
cfm_status cfm_op_linear_pack(int dtype, const float* w, const float* bias, int N, int K, void* pack_ws,
                              size_t* pack_ws_bytes, void* stream) {
  return guarded([&] {
    const int dt = dtype == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16, es = dtype_size(dt);
    if (N <= 0 || K <= 0) fail(CFM_ERR_INVALID_ARG, "N and K must be positive");
    long Kp, Np;
    const size_t need = linear_pack_bytes(dt, N, K, &Kp, &Np);
    if (!pack_ws) {
      if (!pack_ws_bytes) fail(CFM_ERR_INVALID_ARG, "pack_ws_bytes");
      *pack_ws_bytes = need;
      return;
    }
    if (!w) fail(CFM_ERR_INVALID_ARG, "null weight");
    if (K % (16 / es)) fail(CFM_ERR_UNSUPPORTED, "K must be a multiple of 16 bytes");
    if (pack_ws_bytes && *pack_ws_bytes < need) fail(CFM_ERR_WORKSPACE, "pack workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* base = (char*)pack_ws;
    char* bdev = base + Np * Kp * es;
    char* zero = bdev + round_up(Np * 4, 256);
    pack_matrix(dt, w, K, N, K, false, base, Kp, (int)Np, (int)Kp, st);
    HIP_OK(hipMemsetAsync(bdev, 0, (size_t)Np * 4, st));
    if (bias) HIP_OK(hipMemcpyAsync(bdev, bias, (size_t)N * 4, hipMemcpyDeviceToDevice, st));
    HIP_OK(hipMemsetAsync(zero, 0, 4096, st));
    HIP_OK(hipGetLastError());
  });
}

cfm_status cfm_op_linear_packed(int dtype, const void* x, int M, int K, const void* pack_ws, int N, int act, void* y,
                                void* stream) {
  return guarded([&] {
    const int dt = dtype == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16, es = dtype_size(dt);
    if (!x || !pack_ws || !y) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (M < 0 || N <= 0 || K <= 0) fail(CFM_ERR_INVALID_ARG, "bad shape");
    if (K % (16 / es)) fail(CFM_ERR_UNSUPPORTED, "K must be a multiple of 16 bytes");
    long Kp, Np;
    linear_pack_bytes(dt, N, K, &Kp, &Np);
    const char* base = (const char*)pack_ws;
    const char* bdev = base + Np * Kp * es;
    const char* zero = bdev + round_up(Np * 4, 256);
    GemmEpi e = epi_of(act == 1 ? EPI_RELU : act == 2 ? EPI_SWISH : EPI_STORE, (const float*)bdev);
    e.C = y;
    e.ldc = N;
    gemm(dt, x, K, M, K, base, (int)Kp, N, e, zero, (hipStream_t)stream);
    HIP_OK(hipGetLastError());
  });
}

cfm_status cfm_op_linear(int dtype, const void* x, int M, int K, const float* w, const float* bias, int N, int act,
                         void* y, void* pack_ws, size_t* pack_ws_bytes, void* stream) {
  if (!pack_ws) return cfm_op_linear_pack(dtype, w, bias, N, K, nullptr, pack_ws_bytes, stream);
  const cfm_status s = cfm_op_linear_pack(dtype, w, bias, N, K, pack_ws, pack_ws_bytes, stream);
  if (s != CFM_OK) return s;
  return cfm_op_linear_packed(dtype, x, M, K, pack_ws, N, act, y, stream);
}

// ---- ConformerConvolution's middle (conformer_modules.py:164-176) as a kernel-level op --------
}  // extern "C"
namespace {
// GLU over the channel halves [a | gate] of pointwise_conv1's output (nn.functional.glu, dim=1) and
// the pad mask (masked_fill, conformer_modules.py:166-167): g[m][c] = a * sigmoid(gate), 0 on padded frames
template <typename T>
__global__ void glu_mask_kernel(const T* pre, const int32_t* lens, int B, int Tp, int d, T* g) {
  const long n = (long)B * Tp * d;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long m = i / d;
    const int c = (int)(i - m * d);
    const int t = (int)(m % Tp), b = (int)(m / Tp);
    const bool pad = lens && t >= lens[b];
    const float a = ld_f<T>(pre + m * 2 * d + c), gt = ld_f<T>(pre + m * 2 * d + d + c);
    st_f<T>(g + i, pad ? 0.0f : a * sigmoidf_(gt));
  }
}
}  // namespace
extern "C" {

extern "C" size_t cfm_op_conv_glu_dwconv_ws_size(int dtype, int B, int Tp, int d, int K) {
  const int es = dtype == CFM_COMPUTE_FP32 ? 4 : 2;
  const long M = (long)B * Tp;
  return (size_t)(round_up(M * d * es, 256) + round_up(M * d * 4, 256) + round_up((long)d * (K + 6) * 4, 256) + 256);
}

extern "C" cfm_status cfm_op_conv_glu_dwconv(int dtype, const void* pre, const int32_t* lens, int B, int Tp, int d,
                                             int K, const float* dw_w, const float* dw_b, int norm_type,
                                             const float* norm_w, const float* norm_b, const float* bn_mean,
                                             const float* bn_var, void* out, void* ws, size_t ws_bytes, void* stream) {
  return guarded([&] {
    if (!pre || !dw_w || !dw_b || !norm_w || !norm_b || !out || !ws) fail(CFM_ERR_INVALID_ARG, "null argument");
    if (norm_type == 0 && (!bn_mean || !bn_var)) fail(CFM_ERR_INVALID_ARG, "batch_norm needs running statistics");
    if (K < 1 || K % 2 == 0 || B <= 0 || Tp <= 0 || d <= 0) fail(CFM_ERR_INVALID_ARG, "shape");
    if (ws_bytes < cfm_op_conv_glu_dwconv_ws_size(dtype, B, Tp, d, K)) fail(CFM_ERR_WORKSPACE, "workspace too small");
    const int dt = dtype == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16, es = dtype_size(dt);
    const long M = (long)B * Tp;
    hipStream_t st = (hipStream_t)stream;
    char* w = (char*)ws;
    char* G = w;
    float* PN = (float*)(w + round_up(M * d * es, 256));
    float* prm = (float*)((char*)PN + round_up(M * d * 4, 256));
    // depthwise weight (d, 1, K) -> [K][d]; BatchNorm running var -> 1/sqrt(var + eps) (host, as set_weights)
    std::vector<float> hw((size_t)d * K), hv(d, 1.0f), host((size_t)d * (K + 1));
    HIP_OK(hipMemcpyAsync(hw.data(), dw_w, hw.size() * 4, hipMemcpyDeviceToHost, st));
    if (norm_type == 0) HIP_OK(hipMemcpyAsync(hv.data(), bn_var, (size_t)d * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    for (int k = 0; k < K; ++k)
      for (int c = 0; c < d; ++c) host[(size_t)k * d + c] = hw[(size_t)c * K + k];
    for (int c = 0; c < d; ++c) host[(size_t)K * d + c] = 1.0f / std::sqrt(hv[c] + 1e-5f);
    HIP_OK(hipMemcpyAsync(prm, host.data(), host.size() * 4, hipMemcpyHostToDevice, st));
    const dim3 g(1024), b(256);
    if (dt == DT_F32) cfm_launch(glu_mask_kernel<float>, g, b, 0, st, (const float*)pre, lens, B, Tp, d, (float*)G);
    else cfm_launch(glu_mask_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)pre, lens, B, Tp, d, (bf16_t*)G);
    if (norm_type == 0) {
      dwconv_norm_swish(dt, G, B, Tp, d, K, prm, dw_b, bn_mean, prm + (long)K * d, norm_w, norm_b, out, nullptr, st);
    } else {
      dwconv_norm_swish(dt, G, B, Tp, d, K, prm, dw_b, nullptr, nullptr, nullptr, nullptr, nullptr, PN, st);
      layernorm(dt, PN, (int)M, d, norm_w, norm_b, nullptr, nullptr, nullptr, out, 1, st);
    }
    HIP_OK(hipStreamSynchronize(st));   // the host staging vector must outlive the copy
    HIP_OK(hipGetLastError());
  });
}

size_t cfm_op_rel_attention_ws_size(int dtype, int B, int Tp, int H, int dk) {
  const int es = dtype == CFM_COMPUTE_FP32 ? 4 : 2;
  const long dkp = round_up(dk, 16), vt_rows = round_up(dkp, 32), Tpad = round_up(Tp, 32);
  const long M = (long)B * Tp;
  return (size_t)(round_up(M * 3 * H * dkp * es, 256) + round_up((long)B * H * vt_rows * Tpad * es, 256) +
                  round_up((2L * Tp - 1) * H * dkp * es + 64, 256));
}

}  // extern "C"

// head re-layout kernels used only by cfm_op_rel_attention (the encoder writes these layouts
// directly from the QKV / pos GEMM epilogues)
namespace {
template <typename T>
__global__ void pad_heads_kernel(const T* src, long rows, int H, int dk, int dkp, T* dst, long ldd, const float* bias,
                                 float scale) {
  const long n = rows * H * dkp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / (H * dkp);
    const int c = (int)(i % (H * dkp)), hh = c / dkp, dd = c % dkp;
    float v = 0.0f;
    if (dd < dk) v = (ld_f<T>(src + r * H * dk + hh * dk + dd) + (bias ? bias[hh * dk + dd] : 0.0f)) * scale;
    st_f<T>(dst + r * ldd + c, v);
  }
}
template <typename T>
__global__ void vt_kernel(const T* v, int B, int Tp, int H, int dk, int vt_rows, int Tpad, T* vt) {
  const long n = (long)B * H * vt_rows * Tpad;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int t = (int)(i % Tpad);
    const long rest = i / Tpad;
    const int dd = (int)(rest % vt_rows);
    const long bh = rest / vt_rows;
    const int hh = (int)(bh % H), b = (int)(bh / H);
    vt[i] = (dd < dk && t < Tp) ? v[((long)b * Tp + t) * H * dk + hh * dk + dd] : (T)0;
  }
}
template <typename T>
void relayout(const void* q, const void* k, const void* v, const void* p, const float* pos_u, const float* pos_v, int B,
              int Tp, int H, int dk, int dkp, int vt_rows, int Tpad, char* ws, long qk_bytes, long vt_bytes,
              hipStream_t st) {
  const long M = (long)B * Tp;
  T* QK = (T*)ws;
  T* Vt = (T*)(ws + qk_bytes);
  T* P = (T*)(ws + qk_bytes + vt_bytes);
  const dim3 g(1024), b(256);
  const long ld = 3L * H * dkp;
  const float qs = attn_qscale(dk);
  cfm_launch(pad_heads_kernel<T>, g, b, 0, st, (const T*)q, M, H, dk, dkp, QK, ld, pos_u, qs);
  cfm_launch(pad_heads_kernel<T>, g, b, 0, st, (const T*)q, M, H, dk, dkp, QK + (long)H * dkp, ld, pos_v, qs);
  cfm_launch(pad_heads_kernel<T>, g, b, 0, st, (const T*)k, M, H, dk, dkp, QK + 2L * H * dkp, ld,
                     (const float*)nullptr, 1.0f);
  cfm_launch(vt_kernel<T>, g, b, 0, st, (const T*)v, B, Tp, H, dk, vt_rows, Tpad, Vt);
  cfm_launch(pad_heads_kernel<T>, g, b, 0, st, (const T*)p, 2L * Tp - 1, H, dk, dkp, P, (long)H * dkp,
                     (const float*)nullptr, 1.0f);
}
}  // namespace

namespace cfm {
void attn_relayout(int dt, const void* q, const void* k, const void* v, const void* p, const float* pos_u,
                   const float* pos_v, int B, int Tp, int H, int dk, int dkp, int vt_rows, int Tpad, char* ws,
                   long qk_bytes, long vt_bytes, hipStream_t st) {
  if (dt == DT_F32)
    relayout<float>(q, k, v, p, pos_u, pos_v, B, Tp, H, dk, dkp, vt_rows, Tpad, ws, qk_bytes, vt_bytes, st);
  else
    relayout<bf16_t>(q, k, v, p, pos_u, pos_v, B, Tp, H, dk, dkp, vt_rows, Tpad, ws, qk_bytes, vt_bytes, st);
}
}  // namespace cfm

extern "C" cfm_status cfm_op_rel_attention(int dtype, const void* q, const void* k, const void* v, const void* p,
                                           const float* pos_u, const float* pos_v, const int32_t* lens, int B, int Tp,
                                           int H, int dk, int ctx_left, int ctx_right, void* out, void* ws,
                                           void* stream) {
  return guarded([&] {
    if (dk > 128) fail(CFM_ERR_UNSUPPORTED, "head dim > 128");
    const int dt = dtype == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16, es = dtype_size(dt);
    const int dkp = (int)round_up(dk, 16), vt_rows = (int)round_up(dkp, 32), Tpad = (int)round_up(Tp, 32);
    const long M = (long)B * Tp;
    const long qk_bytes = round_up(M * 3 * H * dkp * es, 256);
    const long vt_bytes = round_up((long)B * H * vt_rows * Tpad * es, 256);
    hipStream_t st = (hipStream_t)stream;
    char* w = (char*)ws;
    if (attn_natural_layout(dt, Tp, dkp)) {
      // the encoder's bf16 layout: [q | k | v] rows (heads padded), [u | v] fp32, P padded
      const long ld = 3L * H * dkp;
      const dim3 g(1024), b(256);
      bf16_t* QKV = (bf16_t*)w;
      float* UV = (float*)(w + qk_bytes);
      bf16_t* P = (bf16_t*)(w + qk_bytes + vt_bytes);
      cfm_launch(pad_heads_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)q, M, H, dk, dkp, QKV, ld, (const float*)nullptr, 1.0f);
      cfm_launch(pad_heads_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)k, M, H, dk, dkp, QKV + (long)H * dkp, ld,
                 (const float*)nullptr, 1.0f);
      cfm_launch(pad_heads_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)v, M, H, dk, dkp, QKV + 2L * H * dkp, ld,
                 (const float*)nullptr, 1.0f);
      cfm_launch(pad_heads_kernel<float>, g, b, 0, st, pos_u, 1L, H, dk, dkp, UV, (long)H * dkp, (const float*)nullptr, 1.0f);
      cfm_launch(pad_heads_kernel<float>, g, b, 0, st, pos_v, 1L, H, dk, dkp, UV + (long)H * dkp, (long)H * dkp,
                 (const float*)nullptr, 1.0f);
      cfm_launch(pad_heads_kernel<bf16_t>, g, b, 0, st, (const bf16_t*)p, 2L * Tp - 1, H, dk, dkp, P, (long)H * dkp,
                 (const float*)nullptr, 1.0f);
      rel_pos_attention_natural(QKV, ld, UV, attn_qscale(dk), P, (long)H * dkp, lens, B, Tp, H, dk, dkp, ctx_left,
                                ctx_right, out, (long)H * dk, st);
      HIP_OK(hipGetLastError());
      return;
    }
    attn_relayout(dt, q, k, v, p, pos_u, pos_v, B, Tp, H, dk, dkp, vt_rows, Tpad, (char*)ws, qk_bytes, vt_bytes, st);
    rel_pos_attention(dt, w, 3L * H * dkp, w + qk_bytes, vt_rows, Tpad, w + qk_bytes + vt_bytes, (long)H * dkp, lens,
                      B, Tp, H, dk, dkp, ctx_left, ctx_right, out, (long)H * dk, st);
    HIP_OK(hipGetLastError());
  });
}

// ---- GEMM microbenchmark (tools/gemm_bench.py) ----------------------------------------------
namespace {
__global__ void fill_rand_kernel(uint16_t* p, long n, uint32_t seed, int as_f32) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    const float f = ((x & 0xffffff) / 16777216.0f) * 2.0f - 1.0f;
    if (as_f32) ((float*)p)[i] = f;
    else p[i] = f2bf(f);
  }
}
}  // namespace

extern "C" cfm_status cfm_bench_gemm(int dtype, int tile, int epilogue, int M, int N, int K, int iters,
                                     float* avg_ms) {
  return guarded([&] {
    if (!avg_ms || M <= 0 || N <= 0 || K <= 0 || iters <= 0) fail(CFM_ERR_INVALID_ARG, "bad argument");
    const int dt = dtype == CFM_COMPUTE_FP32 ? DT_F32 : DT_BF16, es = dtype_size(dt);
    const long Kp = round_up(K, GEMM_BK_BYTES / es), Np = round_up(N, GEMM_BN);
    const int epi_mode = epilogue & 15;   // bits 4-5: GEMM probe (see set_gemm_probe)
    const int prev_probe = set_gemm_probe(epilogue >> 4);
    const long Nout = epi_mode == EPI_GLU_MASK ? N : N;
    char *A = nullptr, *W = nullptr, *C = nullptr, *bias = nullptr, *zero = nullptr, *lens = nullptr;
    HIP_OK(hipMalloc(&A, (size_t)M * Kp * es));
    HIP_OK(hipMalloc(&W, (size_t)Np * 2 * Kp * es));
    HIP_OK(hipMalloc(&C, (size_t)M * Np * 4));
    HIP_OK(hipMalloc(&bias, (size_t)Np * 2 * 4));
    HIP_OK(hipMalloc(&zero, 4096));
    HIP_OK(hipMalloc(&lens, 4096));
    HIP_OK(hipMemset(zero, 0, 4096));
    HIP_OK(hipMemset(bias, 0, (size_t)Np * 2 * 4));
    HIP_OK(hipMemset(C, 0, (size_t)M * Np * 4));
    std::vector<int32_t> hl(1024, 1 << 30);
    HIP_OK(hipMemcpy(lens, hl.data(), 4096, hipMemcpyHostToDevice));
    cfm_launch(fill_rand_kernel, dim3(1024), dim3(256), 0, 0, (uint16_t*)A, (long)M * Kp * (es / 2), 1u, 0);
    cfm_launch(fill_rand_kernel, dim3(1024), dim3(256), 0, 0, (uint16_t*)W, (long)Np * 2 * Kp * (es / 2), 2u, 0);
    GemmEpi e = epi_of(epi_mode, (const float*)bias, 1.0f);
    e.C = C; e.ldc = Nout; e.X = (float*)C; e.ldx = Nout; e.lens = (const int32_t*)lens; e.Tp = 1 << 20;
    e.Vt = C; e.H = 1; e.dkp = 64; e.vt_rows = 64; e.Tpad = M; e.qk_cols = 2 * N / 3; e.uv = (const float*)bias;
    e.qscale = 1.0f;
    if (epi_mode == EPI_QKV) e.ldc = 4 * N / 3;
    const int prev = set_gemm_tile_override(tile);
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    for (int i = 0; i < 3; ++i) gemm(dt, A, Kp, M, K, W, (int)Kp, N, e, zero, 0);
    HIP_OK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) gemm(dt, A, Kp, M, K, W, (int)Kp, N, e, zero, 0);
    HIP_OK(hipEventRecord(e1, 0));
    HIP_OK(hipEventSynchronize(e1));
    set_gemm_tile_override(prev);
    set_gemm_probe(prev_probe);
    float ms = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    *avg_ms = ms / iters;
    (void)hipEventDestroy(e0); (void)hipEventDestroy(e1);
    (void)hipFree(A); (void)hipFree(W); (void)hipFree(C); (void)hipFree(bias); (void)hipFree(zero); (void)hipFree(lens);
    HIP_OK(hipGetLastError());
  });
}
