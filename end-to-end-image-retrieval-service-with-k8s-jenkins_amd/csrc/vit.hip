// vit.hip — ViT-MSN embedding model: weights, workspace and the launch sequence
// behind rc_embed (replaces embedding/main.py:97-114's ViTImageProcessor +
// ViTMSNModel + CLS extraction).
//
// HBM layout per model (bf16 GEMM operands, bf16 residual stream under the LayerNorm fold):
//   weights   W_qkv [3H][H] (q,k,v rows concatenated), W_o [H][H], W_fc1 [MLP][H],
//             W_fc2 [H][MLP] — bf16, nn.Linear [out][in]; W_patch [H][P·P·3] bf16 with
//             K ordered (ky, kx, c) for the implicit-GEMM patch embedding;
//             biases / LayerNorm params / cls / pos — f32
//   workspace (sized for max_batch images, rows padded to the GEMM tile):
//             residual stream: under the LayerNorm fold ln = RNE_bf16(x) [Mp][H] with
//             ln_stats f32 [Mp][LN_PARTS][2]; without it
//             hidden f32 [Mp][H] and ln bf16 [Mp][H] = LayerNorm output; qkv bf16
//             [Mp][3H], attn bf16 [Mp][H], mlp bf16 [Mp][MLP]
#include <algorithm>
#include <cmath>
#include <map>
#include <string>
#include <vector>

#include "gemm.h"
#include "resample.h"
#include "vit_kernels.h"

using namespace rc;

namespace {

int round_up(int x, int m) { return (x + m - 1) / m * m; }

struct DeviceCoeffs {
    int ksize = 0;
    int *bounds = nullptr;
    int *coef = nullptr;
    int first = 0, last = 0;  // used source range [first, last)
};

struct Layer {
    uint16_t *w_qkv = nullptr, *w_o = nullptr, *w_fc1 = nullptr, *w_fc2 = nullptr;
    float *b_qkv = nullptr, *b_o = nullptr, *b_fc1 = nullptr, *b_fc2 = nullptr;
    float *ln1_w = nullptr, *ln1_b = nullptr, *ln2_w = nullptr, *ln2_b = nullptr;
    // LayerNorm folded into QKV / fc1 (vit_kernels.h "LayerNorm fold"): W′ = W·diag(γ) in
    // bf16, c = Σ_k W′ (of the bf16 values), b′ = b + W·β
    uint16_t *w_qkv_f = nullptr, *w_fc1_f = nullptr;
    float *b_qkv_f = nullptr, *c_qkv = nullptr, *b_fc1_f = nullptr, *c_fc1 = nullptr;
};

constexpr int kMaxParts = 4;

// T_GEMM: every GEMM; T_QKV / T_OPROJ / T_FC1 / T_FC2: that projection's full-batch
// launches (M = images x 197 rows), each priced on its own in the bench
enum TimerId { T_GEMM = 0, T_FC1 = 1, T_ATTN = 2, T_LN = 3, T_PRE = 4, T_QKV = 5, T_OPROJ = 6, T_FC2 = 7, T_COUNT = 8 };

}  // namespace

struct rc_model {
    std::mutex mu;
    int device = 0;
    rc_vit_config cfg{};
    int tokens = 0, npatch = 0, kpatch = 0;
    std::map<std::string, std::vector<int64_t>> shapes;  // expected tensors
    std::map<std::string, std::vector<float>> host;      // staged until finalize
    bool ready = false;
    std::vector<void *> allocs;
    // device weights
    uint16_t *w_patch = nullptr;
    float *b_patch = nullptr, *cls = nullptr, *pos = nullptr, *lnf_w = nullptr, *lnf_b = nullptr;
    std::vector<Layer> layers;
    // preprocessing
    int resample = RC_RESAMPLE_BICUBIC;
    double rescale = 1.0 / 255.0;
    float mean[3] = {0.485f, 0.456f, 0.406f}, std_[3] = {0.229f, 0.224f, 0.225f};
    float *lut = nullptr;          // [3][256] f32: rescale→normalize of each u8 (pixel_values)
    float pre_a[3] = {}, pre_b[3] = {};  // the patch GEMM's A operand: bf16(fma(u, pre_a[c], pre_b[c]))
    std::map<std::pair<int, int>, DeviceCoeffs> coeff_cache;  // (in, out) → coeffs
    // workspace
    int Mp = 0;
    uint16_t *ln = nullptr, *qkv = nullptr, *attn = nullptr, *mlp = nullptr;
    float *hidden = nullptr;
    float *ln_stats = nullptr;     // [Mp][LN_PARTS][2] LayerNorm-fold partials (per 64-column block: mean, M2)
    bool ln_fold = true;           // rc_model_set_ln_fold: LN folded into QKV / fc1 for M > 256 rows
    // last layer on the CLS rows only (compact [max_batch + pad][·] streams)
    bool cls_only_last = true;     // rc_model_set_last_layer
    float *cls_hidden = nullptr, *cls_stats = nullptr;
    float *cls_part = nullptr;     // split-K partials of the CLS-row fc2 [SKINNY_KS][Cp][H]
    uint16_t *cls_ln = nullptr, *cls_attn = nullptr, *cls_mlp = nullptr;
    uint8_t *resized = nullptr, *resize_tmp = nullptr;
    size_t resize_tmp_bytes = 0;
    KernelTimer timers[T_COUNT];
    int gemm_variant = GEMM_AUTO;  // diagnostic builds only: rc_diag_set_gemm_variant
    int attn_form = 2;             // attention_v2_kernel; diag builds: 3 = attention_v3_kernel (A/B: v3 lost, 92 vs 75 us)
    int ncu = 256;                 // compute units (persistent grids)
    int split = 2;                 // batch parts encoded concurrently (rc_model_set_parts);
                                   // 2 beats 3 and 4 by 1-2 % at batch 256 (profiles/r01j_ab_parts.jsonl)
    int split_min = 32;            // fewest images per part
    hipStream_t sp[4] = {};        // streams of parts 1..3 (part 0 runs on the caller's stream)
    hipEvent_t ev_fork = nullptr, ev_join[4] = {};
    // Batch-1 launch chains replayed as HIP graphs (rc_model_set_graphs): one instantiated graph per
    // (images, raw, normed) buffer triple, least recently used evicted past kMaxGraphs.  The graph
    // bakes every pointer and setting into its kernel arguments, so every setter clears the cache.
    struct EmbedGraph {
        const uint8_t *images;
        float *raw, *normed;
        hipGraphExec_t exec;
        uint64_t last;
    };
    static constexpr int kMaxGraphs = 8;
    bool use_graphs = true;
    std::vector<EmbedGraph> graphs;
    uint64_t graph_tick = 0;
    // misses in a row, and the last missed triple: once kMaxGraphs calls in a row missed (the
    // caller's buffers churn), only a triple that misses twice in a row is captured
    int graph_miss_streak = 0;
    EmbedGraph last_miss{};
    void clear_graphs() {
        for (auto &g : graphs) (void)hipGraphExecDestroy(g.exec);
        graphs.clear();
        graph_miss_streak = 0;
        last_miss = EmbedGraph{};
    }

    void *alloc(size_t bytes) {
        void *p = dmalloc(bytes);
        allocs.push_back(p);
        return p;
    }
    ~rc_model() {
        clear_graphs();
        for (auto &t : timers) t.destroy();
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        for (auto &e : ev_join)
            if (e) (void)hipEventDestroy(e);
        for (auto &q : sp)
            if (q) (void)hipStreamDestroy(q);
        for (void *p : allocs) dfree(p);
        dfree(resize_tmp);
    }
};

namespace {

std::string canonical_name(std::string n) {
    if (n.rfind("vit.", 0) == 0) n = n.substr(4);
    if (n.rfind("layers.", 0) == 0) n = "encoder.layer." + n.substr(7);
    const std::pair<const char *, const char *> ren[] = {
        {"attention.q_proj", "attention.attention.query"}, {"attention.k_proj", "attention.attention.key"},
        {"attention.v_proj", "attention.attention.value"}, {"attention.o_proj", "attention.output.dense"},
        {"mlp.fc1", "intermediate.dense"},                 {"mlp.fc2", "output.dense"},
    };
    for (auto &r : ren) {
        const size_t p = n.find(r.first);
        if (p != std::string::npos) {
            n.replace(p, std::strlen(r.first), r.second);
            break;
        }
    }
    return n;
}

void build_shapes(rc_model *m) {
    const auto &c = m->cfg;
    const int64_t H = c.hidden, F = c.mlp;
    auto &s = m->shapes;
    s["embeddings.cls_token"] = {1, 1, H};
    s["embeddings.position_embeddings"] = {1, m->tokens, H};
    s["embeddings.patch_embeddings.projection.weight"] = {H, 3, c.patch, c.patch};
    s["embeddings.patch_embeddings.projection.bias"] = {H};
    for (int i = 0; i < c.layers; ++i) {
        const std::string p = "encoder.layer." + std::to_string(i) + ".";
        for (const char *nm : {"query", "key", "value"}) {
            s[p + "attention.attention." + nm + ".weight"] = {H, H};
            s[p + "attention.attention." + nm + ".bias"] = {H};
        }
        s[p + "attention.output.dense.weight"] = {H, H};
        s[p + "attention.output.dense.bias"] = {H};
        s[p + "intermediate.dense.weight"] = {F, H};
        s[p + "intermediate.dense.bias"] = {F};
        s[p + "output.dense.weight"] = {H, F};
        s[p + "output.dense.bias"] = {H};
        for (const char *nm : {"layernorm_before", "layernorm_after"}) {
            s[p + nm + ".weight"] = {H};
            s[p + nm + ".bias"] = {H};
        }
    }
    s["layernorm.weight"] = {H};
    s["layernorm.bias"] = {H};
}

int64_t numel_of(const std::vector<int64_t> &sh) {
    int64_t n = 1;
    for (auto d : sh) n *= d;
    return n;
}

float *upload_f32(rc_model *m, const std::vector<float> &v) {
    float *d = (float *)m->alloc(v.size() * sizeof(float));
    RC_HIP(hipMemcpy(d, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice));
    return d;
}

uint16_t *upload_bf16(rc_model *m, const std::vector<const std::vector<float> *> &parts) {
    size_t n = 0;
    for (auto *p : parts) n += p->size();
    std::vector<uint16_t> h(n);
    size_t o = 0;
    for (auto *p : parts)
        for (float f : *p) h[o++] = host_f2bf(f);
    uint16_t *d = (uint16_t *)m->alloc(n * sizeof(uint16_t));
    RC_HIP(hipMemcpy(d, h.data(), n * sizeof(uint16_t), hipMemcpyHostToDevice));
    return d;
}

float bits_f32(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
uint32_t f32_bits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

// The patch GEMM converts a byte u of channel c as bf16(fmaf(u, a_c, b_c)).  Find f32 (a_c, b_c)
// near 1 / (rescale⁻¹·std) and −mean / std for which that equals, for ALL 256 values of u, the
// bf16 of ViTImageProcessor's f32 value h(u) (exact for the ImageNet parameters at ±0 ulp; the
// search covers ±16 ulp of each).  Parameters with no exact pair are refused rather than
// approximated.
bool exact_affine(const float *h, double a0, double b0, float *a_out, float *b_out) {
    const float a = (float)a0, b = (float)b0;
    for (int da = 0; da <= 32; ++da)
        for (int db = 0; db <= 32; ++db) {
            const float aa = bits_f32(f32_bits(a) + (uint32_t)((da & 1) ? -(da + 1) / 2 : da / 2));
            const float bb = bits_f32(f32_bits(b) + (uint32_t)((db & 1) ? -(db + 1) / 2 : db / 2));
            bool ok = true;
            for (int u = 0; u < 256 && ok; ++u) ok = host_f2bf(std::fmaf((float)u, aa, bb)) == host_f2bf(h[u]);
            if (ok) {
                *a_out = aa;
                *b_out = bb;
                return true;
            }
        }
    return false;
}

void build_lut(rc_model *m) {
    float h[3 * 256];
    for (int c = 0; c < 3; ++c)
        for (int u = 0; u < 256; ++u) {
            // transformers rescale: u8 -> f64 * factor -> f32; normalize in f32: (x - mean) / std
            const float x = (float)((double)u * m->rescale);
            h[c * 256 + u] = (x - m->mean[c]) / m->std_[c];
        }
    float pa[3], pb[3];
    for (int c = 0; c < 3; ++c)
        RC_REQUIRE(exact_affine(h + c * 256, m->rescale / m->std_[c], -(double)m->mean[c] / m->std_[c], &pa[c], &pb[c]),
                   RC_ERR_UNSUPPORTED,
                   "preprocess parameters: no f32 affine form reproduces ViTImageProcessor's bf16-rounded values "
                   "for every byte of channel " + std::to_string(c));
    if (!m->lut) m->lut = (float *)m->alloc(sizeof(h));
    RC_HIP(hipMemcpy(m->lut, h, sizeof(h), hipMemcpyHostToDevice));
    for (int c = 0; c < 3; ++c) {
        m->pre_a[c] = pa[c];
        m->pre_b[c] = pb[c];
    }
}

// LayerNorm fold of one nn.Linear W [N][K] after LayerNorm(γ, β) (vit_kernels.h):
// W′ = bf16(W·diag(γ)), c_n = Σ_k W′[n][k] (the bf16 values the MFMAs multiply,
// summed in f64), b′_n = b_n + Σ_k W[n][k]·β_k (f64, from the f32 weights).
void fold_layernorm(rc_model *m, const std::vector<float> &W, const std::vector<float> &b, const std::vector<float> &g,
                    const std::vector<float> &beta, uint16_t **w_out, float **b_out, float **c_out) {
    const size_t K = g.size(), N = b.size();
    std::vector<float> wf(N * K), bf(N), cf(N);
    for (size_t n = 0; n < N; ++n) {
        double cs = 0.0, bs = b[n];
        for (size_t k = 0; k < K; ++k) {
            const float w = W[n * K + k] * g[k];
            uint32_t u;
            const uint16_t hb = host_f2bf(w);
            u = (uint32_t)hb << 16;
            float wr;
            std::memcpy(&wr, &u, 4);
            wf[n * K + k] = w;
            cs += wr;
            bs += (double)W[n * K + k] * beta[k];
        }
        cf[n] = (float)cs;
        bf[n] = (float)bs;
    }
    *w_out = upload_bf16(m, {&wf});
    *b_out = upload_f32(m, bf);
    *c_out = upload_f32(m, cf);
}

const DeviceCoeffs &get_coeffs(rc_model *m, int in_size, int out_size) {
    auto key = std::make_pair(in_size * 8 + m->resample, out_size);
    auto it = m->coeff_cache.find(key);
    if (it != m->coeff_cache.end()) return it->second;
    ResampleCoeffs c = precompute_coeffs(in_size, out_size, m->resample);
    DeviceCoeffs d;
    d.ksize = c.ksize;
    d.bounds = (int *)m->alloc(c.bounds.size() * sizeof(int));
    d.coef = (int *)m->alloc(c.coef.size() * sizeof(int));
    RC_HIP(hipMemcpy(d.bounds, c.bounds.data(), c.bounds.size() * sizeof(int), hipMemcpyHostToDevice));
    RC_HIP(hipMemcpy(d.coef, c.coef.data(), c.coef.size() * sizeof(int), hipMemcpyHostToDevice));
    d.first = c.bounds[0];
    d.last = c.bounds[2 * (out_size - 1)] + c.bounds[2 * (out_size - 1) + 1];
    return m->coeff_cache.emplace(key, d).first->second;
}

unsigned grid_for(int64_t work, int per_block = 256) {
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>((work + per_block - 1) / per_block, 256 * 16));
}

// Pillow-exact resize of n images (h, w) → (S, S) into m->resized; returns the source to use.
// As ImagingResampleInner: a pass runs only if its axis changes; the horizontal
// pass covers just the source rows the vertical pass reads, whose bounds are then
// taken relative to the first of them.
const uint8_t *resize_batch(rc_model *m, const uint8_t *images, int n, int h, int w, hipStream_t s) {
    const int S = m->cfg.image_size;
    if (h == S && w == S) return images;
    const bool need_h = w != S, need_v = h != S;
    const DeviceCoeffs &cv = get_coeffs(m, h, S);
    const DeviceCoeffs &ch = get_coeffs(m, w, S);
    const uint8_t *cur = images;
    int cur_h = h;
    if (need_h) {
        const int y0 = need_v ? cv.first : 0, Hs = need_v ? cv.last - cv.first : h;
        const size_t bytes = (size_t)n * Hs * S * 3;
        if (bytes > m->resize_tmp_bytes) {
            RC_HIP(hipStreamSynchronize(s));
            dfree(m->resize_tmp);
            m->resize_tmp = nullptr;
            m->resize_tmp = (uint8_t *)dmalloc(bytes);
            m->resize_tmp_bytes = bytes;
        }
        hipLaunchKernelGGL(resize_h_kernel, dim3(grid_for((int64_t)n * Hs * S)), dim3(256), 0, s, images, h, w, y0, Hs,
                           m->resize_tmp, S, ch.bounds, ch.coef, ch.ksize, n);
        RC_LAUNCH_CHECK();
        cur = m->resize_tmp;
        cur_h = Hs;
        if (!need_v) {
            RC_HIP(hipMemcpyAsync(m->resized, cur, (size_t)n * S * S * 3, hipMemcpyDeviceToDevice, s));
            return m->resized;
        }
    }
    const int *vb = cv.bounds;
    if (need_h && cv.first != 0) {
        auto key = std::make_pair(-(h * 8 + m->resample), S);  // shifted copy of the vertical bounds
        auto it = m->coeff_cache.find(key);
        if (it == m->coeff_cache.end()) {
            ResampleCoeffs c = precompute_coeffs(h, S, m->resample);
            for (int i = 0; i < S; ++i) c.bounds[2 * i] -= cv.first;
            DeviceCoeffs d = cv;
            d.bounds = (int *)m->alloc(c.bounds.size() * sizeof(int));
            RC_HIP(hipMemcpy(d.bounds, c.bounds.data(), c.bounds.size() * sizeof(int), hipMemcpyHostToDevice));
            it = m->coeff_cache.emplace(key, d).first;
        }
        vb = it->second.bounds;
    }
    const int cur_w = need_h ? S : w;
    hipLaunchKernelGGL(resize_v_kernel, dim3(grid_for((int64_t)n * S * cur_w)), dim3(256), 0, s, cur, cur_h, cur_w,
                       m->resized, S, vb, cv.coef, cv.ksize, n);
    RC_LAUNCH_CHECK();
    return m->resized;
}

#if defined(RC_GEMM_ABLATION)
// Diagnostic builds: the A/B kernel for a full-batch projection.  The residual producers
// (O-proj, fc2; auto = two-workgroup / ping-pong) take GEMM_PINGPONG / GEMM_W2 / GEMM_PP_IMG;
// ping-pong ablations (100 + ABL) apply where auto picks the 256-row ping-pong kernel.
int diag_variant(const GemmArgs &a, int variant, bool patch_epilogue, bool ln_epilogue) {
    if (variant == GEMM_AUTO) return variant;
    const int pick = gemm_pick(a, GEMM_AUTO, patch_epilogue, ln_epilogue);
    const bool producer = a.row_step > 0 && pick != GEMM_SKINNY;  // O-proj / fc2 of a full batch
    if (producer && (variant == GEMM_PINGPONG || variant == GEMM_W2 || variant == GEMM_PP_IMG)) return variant;
    if (producer && variant == 11) return a.K <= 768 ? GEMM_W2 : GEMM_PP_IMG;  // O-proj two-workgroup, fc2 image-aligned
    if (producer && variant == 12) return a.K <= 768 ? GEMM_W2 : GEMM_PINGPONG;  // = auto (rounds 4 and 5)
    if (producer && variant == 13) return a.K <= 768 ? 300 : GEMM_PINGPONG;      // O-proj on 128-row W2 tiles only
    if (producer && variant == 14) return GEMM_W2;                                // fc2 on the two-workgroup kernel too
    // residual epilogues with nontemporal reads / stores / both: O-proj (W2 160-row tiles) 18-20,
    // fc2 (ping-pong) 21-23
    if (producer && variant >= 18 && variant <= 20) return a.K <= 768 ? 300 + (variant - 17) : GEMM_AUTO;
    if (producer && variant >= 21 && variant <= 23) return a.K > 768 ? 153 + (variant - 21) : GEMM_AUTO;
    // the A operand's DMA nontemporal: 24 fc2, 25 O-proj, 26 both
    if (producer && (variant == 24 || variant == 26) && a.K > 768) return 156;
    if (producer && (variant == 25 || variant == 26) && a.K <= 768) return 304;
    // LayerNorm-fold consumers of a full batch on the two-workgroup kernel: 15 fc1, 16 QKV, 17 both
    if (ln_epilogue && pick == GEMM_PINGPONG &&
        (variant == 17 || (variant == 15 && a.N == 3072) || (variant == 16 && a.N != 3072)))
        return GEMM_W2;
    if (pick == GEMM_PINGPONG && variant >= 100 && variant < 200) return variant;
    return GEMM_AUTO;
}
#endif

// role: T_QKV / T_OPROJ / T_FC1 / T_FC2 (its own timer besides T_GEMM), or -1
template <int EPI>
void gemm(rc_model *m, const GemmArgs &a, hipStream_t s, int role = -1) {
    const double flops = 2.0 * a.M * a.N * a.K;
    const int t0 = m->timers[T_GEMM].begin(s);
    const int t1 = role >= 0 ? m->timers[role].begin(s) : -1;
    int variant = GEMM_AUTO;
#if defined(RC_GEMM_ABLATION)
    variant = diag_variant(a, m->gemm_variant, epi_patch(EPI), epi_ln(EPI));
#endif
    launch_gemm<EPI>(a, variant, s);
    if (role >= 0) m->timers[role].end(t1, s, flops);
    m->timers[T_GEMM].end(t0, s, flops);
}

// residual-stream producer GEMM (O-proj, fc2): f32 stream, or bf16 under the fold
void resid_gemm(rc_model *m, const GemmArgs &a, hipStream_t s, int role) {
    if (a.resid_bf16) gemm<EPI_RESID_BF16>(m, a, s, role);
    else gemm<EPI_RESID_F32>(m, a, s, role);
}

void layernorm(rc_model *m, const float *x, const float *g, const float *b, uint16_t *y, int M, hipStream_t s) {
    const int t = m->timers[T_LN].begin(s);
    hipLaunchKernelGGL(layernorm_kernel<3>, dim3((M + 3) / 4), dim3(256), 0, s, x, g, b, y, M, m->cfg.ln_eps);
    RC_LAUNCH_CHECK();
    m->timers[T_LN].end(t, s, (double)M * m->cfg.hidden * 6.0);
}

// Last encoder layer after its QKV GEMM, for the CLS rows only (see
// attention_cls_kernel): gather the n CLS rows of the residual stream into
// cls_hidden[i0 ..], CLS-query attention, then O-proj (+residual), LN2, fc1+GELU
// and fc2 (+residual) as M = n GEMMs on the compact rows.  The kernels are the
// full-batch ones (a GEMM row's result does not depend on M), so a CLS row gets
// the same arithmetic as in the full layer except attention's summation order.
void last_layer_cls(rc_model *m, const Layer &L, int i0, int n, const uint16_t *qkv, const float *hidden,
                    const uint16_t *hi, const float *st_rows, float scale, hipStream_t s) {
    const auto &c = m->cfg;
    const int H = c.hidden, T = m->tokens;
    float *hc = m->cls_hidden + (int64_t)i0 * H;
    uint16_t *ac = m->cls_attn + (int64_t)i0 * H, *lc = m->cls_ln + (int64_t)i0 * H;
    uint16_t *mc = m->cls_mlp + (int64_t)i0 * c.mlp;
    // LayerNorm fold: the QKV GEMM before this produced K and V only; Q is needed for the
    // CLS rows alone, from their bf16 rows and statistics gathered compact (same arithmetic
    // as the full QKV GEMM: the skinny / tiled kernels give a row the same bits at any M)
    const bool q_cls = m->ln_fold && hi != nullptr;
    float *cst = m->cls_stats + (int64_t)i0 * LN_STRIDE;
    uint16_t *qc = m->cls_mlp + (int64_t)i0 * c.mlp;  // [n][H] compact queries (fc1 overwrites it later)
    hipLaunchKernelGGL(gather_cls_kernel, dim3(n), dim3(H / 4), 0, s, hidden, hi, T, hc, q_cls ? lc : nullptr,
                       st_rows, cst);
    RC_LAUNCH_CHECK();
    if (q_cls) {
        GemmArgs q{lc, L.w_qkv_f, L.b_qkv_f, n, H, H, qc, nullptr, nullptr, 1};
        q.ln_c = L.c_qkv;
        q.ln_stats = cst;
        q.ln_eps = c.ln_eps;
        gemm<EPI_BF16_LN>(m, q, s);
    }
    const int ta = m->timers[T_ATTN].begin(s);
    const int items = n * c.heads;
    hipLaunchKernelGGL(attention_cls_kernel, dim3((items + 3) / 4), dim3(256), 0, s, qkv, ac, T, c.heads, items,
                       scale * 1.4426950408889634f, q_cls ? qc : nullptr);
    RC_LAUNCH_CHECK();
    m->timers[T_ATTN].end(ta, s, 4.0 * items * (double)T * (H / c.heads));
    GemmArgs o{ac, L.w_o, L.b_o, n, H, H, nullptr, hc, nullptr, 1};
    if (m->ln_fold) {  // LN2 folded into fc1, as in the other layers
        float *st = m->cls_stats + (int64_t)i0 * LN_STRIDE;
        o.ln_x = lc;
        o.ln_stats = st;
        gemm<EPI_RESID_F32>(m, o, s);
        GemmArgs f{lc, L.w_fc1_f, L.b_fc1_f, n, c.mlp, H, mc, nullptr, nullptr, 1};
        f.ln_c = L.c_fc1;
        f.ln_stats = st;
        f.ln_eps = c.ln_eps;
        gemm<EPI_GELU_BF16_LN>(m, f, s);
    } else {
        gemm<EPI_RESID_F32>(m, o, s);
        layernorm(m, hc, L.ln2_w, L.ln2_b, lc, n, s);
        gemm<EPI_GELU_BF16>(m, GemmArgs{lc, L.w_fc1, L.b_fc1, n, c.mlp, H, mc, nullptr, nullptr, 1}, s);
    }
    {  // fc2 (K = 3072) split over K: the plain skinny kernel's K chain is latency-bound
        const GemmArgs f2{mc, L.w_fc2, L.b_fc2, n, H, c.mlp, nullptr, hc, nullptr, 1};
        const double flops = 2.0 * f2.M * f2.N * f2.K;
        const int t0 = m->timers[T_GEMM].begin(s);
        launch_skinny_splitk_resid(f2, m->cls_part + (int64_t)i0 * SKINNY_KS * H, s);  // per part: disjoint
        m->timers[T_GEMM].end(t0, s, flops);
    }
}

// Encoder for images [i0, i0 + n) of the batch (u8 S x S x 3 images at `images`,
// already resized): CLS + pos, implicit-GEMM patch embedding, 12 layers, final LN
// on the CLS rows.  Every buffer is addressed from the first image's rows, so two
// parts of a batch can run on two streams at once (GEMM A tiles may read up to 255
// rows past a part's last row; those rows are allocated and their results are
// never stored).
void encode(rc_model *m, const uint8_t *images, int i0, int n, float *raw, float *normed, hipStream_t s) {
    const auto &c = m->cfg;
    const int H = c.hidden, T = m->tokens, M = n * T, S = c.image_size;
    const int64_t r0 = (int64_t)i0 * T;  // first token row of this part
    float *hidden = m->hidden + r0 * H;
    uint16_t *ln = m->ln + r0 * H, *qkv = m->qkv + r0 * 3 * H, *attn = m->attn + r0 * H;
    uint16_t *mlp = m->mlp + r0 * c.mlp;
    // LayerNorm fold (vit_kernels.h): every producer of the residual stream also writes
    // bf16(x) into `ln` and per-tile partials into `st`; QKV and fc1 apply the norm in
    // their epilogues.  The same arithmetic at every batch size (skinny GEMMs for
    // M <= 256 included), so an image's embedding does not depend on its batch.
    const bool fold = m->ln_fold;
    float *st = m->ln_stats + r0 * LN_STRIDE;
    auto produce = [&](GemmArgs a, bool emit) {
        if (fold) {  // the residual stream is `ln` itself (bf16)
            a.ln_x = ln;
            a.resid_bf16 = true;
            a.ln_stats = emit ? st : nullptr;
        }
        return a;
    };
    // 2. embeddings: CLS + pos, patch GEMM (+bias +pos) into the residual stream
    hipLaunchKernelGGL(cls_init_kernel, dim3(n), dim3(256), 0, s, hidden, T, H, m->cls, m->pos, fold ? ln : nullptr,
                       fold ? st : nullptr);
    RC_LAUNCH_CHECK();
    {
        GemmArgs a = produce(GemmArgs{nullptr, m->w_patch, m->b_patch, n * m->npatch, H, m->kpatch, nullptr, hidden, m->pos,
                                      T}, true);
        a.img = images + (int64_t)i0 * S * S * 3;
        for (int c = 0; c < 3; ++c) {
            a.pre_a[c] = m->pre_a[c];
            a.pre_b[c] = m->pre_b[c];
        }
        a.img_size = S;
        const int t0 = m->timers[T_GEMM].begin(s);
        launch_patch_gemm(a, s);
        m->timers[T_GEMM].end(t0, s, 2.0 * a.M * a.N * a.K);
    }
    // 3. encoder layers
    const float scale = 1.0f / std::sqrt((float)(H / c.heads));
    for (int l = 0; l < c.layers; ++l) {
        const Layer &L = m->layers[l];
        if (fold) {
            // the CLS-only last layer needs Q on the CLS rows alone (last_layer_cls): K and V
            // here, into their columns of the qkv rows
            const bool kv_only = m->cls_only_last && l == c.layers - 1;
            const int64_t q0 = kv_only ? H : 0;
            GemmArgs a{ln, L.w_qkv_f + q0 * H, L.b_qkv_f + q0, M, 3 * H - (int)q0, H, qkv + q0, nullptr, nullptr, T};
            a.ldc = 3 * H;
            a.ln_c = L.c_qkv + q0;
            a.ln_stats = st;
            a.ln_eps = c.ln_eps;
            gemm<EPI_BF16_LN>(m, a, s, kv_only ? -1 : T_QKV);
        } else {
            layernorm(m, hidden, L.ln1_w, L.ln1_b, ln, M, s);
            gemm<EPI_BF16>(m, GemmArgs{ln, L.w_qkv, L.b_qkv, M, 3 * H, H, qkv, nullptr, nullptr, T}, s, T_QKV);
        }
        if (m->cls_only_last && l == c.layers - 1) {
            last_layer_cls(m, L, i0, n, qkv, hidden, fold ? ln : nullptr, st, scale, s);
            break;
        }
        const int ta = m->timers[T_ATTN].begin(s);
        const int items = n * c.heads;
        // fewer items than CUs: each item's query tiles split over 4 blocks (a lone image: 48 blocks)
        const int qsplit = items < m->ncu ? 4 : 1;
#if defined(RC_GEMM_ABLATION)
        if (m->attn_form == 3) {  // persistent: two blocks per CU walk the (image, head) items
            const int nb = std::min(items, 2 * m->ncu);
            hipLaunchKernelGGL(attention_v3_kernel<197>, dim3(nb), dim3(256), 0, s, qkv, attn, T, c.heads, items,
                               scale * 1.4426950408889634f);
        } else if (m->attn_form == 4 && T == 197) {  // v2, co-resident blocks staggered by ~6 us
            hipLaunchKernelGGL((attention_v2_kernel<197, 600>), dim3(items * qsplit), dim3(256), 0, s, qkv, attn, T, c.heads,
                               scale * 1.4426950408889634f, qsplit);
        } else if (m->attn_form == 6 && T == 197) {  // v2 with the default-policy K/V DMA (rounds 1-5)
            hipLaunchKernelGGL((attention_v2_kernel<197, 0, 0>), dim3(items * qsplit), dim3(256), 0, s, qkv, attn, T, c.heads,
                               scale * 1.4426950408889634f, qsplit);
        } else if (m->attn_form == 5 && T == 197) {  // ~3 us
            hipLaunchKernelGGL((attention_v2_kernel<197, 300>), dim3(items * qsplit), dim3(256), 0, s, qkv, attn, T, c.heads,
                               scale * 1.4426950408889634f, qsplit);
        } else
#endif
        if (T == 197) {
            hipLaunchKernelGGL(attention_v2_kernel<197>, dim3(items * qsplit), dim3(256), 0, s, qkv, attn, T, c.heads,
                               scale * 1.4426950408889634f, qsplit);
        } else {
            hipLaunchKernelGGL(attention_v2_kernel<0>, dim3(items * qsplit), dim3(256), 0, s, qkv, attn, T, c.heads,
                               scale * 1.4426950408889634f, qsplit);
        }
        RC_LAUNCH_CHECK();
        m->timers[T_ATTN].end(ta, s, 4.0 * n * c.heads * (double)T * T * (H / c.heads));
        {
            GemmArgs o = produce(GemmArgs{attn, L.w_o, L.b_o, M, H, H, nullptr, hidden, nullptr, T}, true);
            o.row_step = T;  // rows per image (diagnostic builds: image-aligned tiles, gemm_pp_kernel<.., 224>)
            resid_gemm(m, o, s, T_OPROJ);
        }
        if (fold) {
            GemmArgs a{ln, L.w_fc1_f, L.b_fc1_f, M, c.mlp, H, mlp, nullptr, nullptr, T};
            a.ln_c = L.c_fc1;
            a.ln_stats = st;
            a.ln_eps = c.ln_eps;
            gemm<EPI_GELU_BF16_LN>(m, a, s, T_FC1);
        } else {
            layernorm(m, hidden, L.ln2_w, L.ln2_b, ln, M, s);
            gemm<EPI_GELU_BF16>(m, GemmArgs{ln, L.w_fc1, L.b_fc1, M, c.mlp, H, mlp, nullptr, nullptr, T}, s, T_FC1);
        }
        // the last layer's fc2 feeds only the final LN of the CLS rows (cls_final_kernel)
        {
            GemmArgs f2 = produce(GemmArgs{mlp, L.w_fc2, L.b_fc2, M, H, c.mlp, nullptr, hidden, nullptr, T}, l + 1 < c.layers);
            f2.row_step = T;
            resid_gemm(m, f2, s, T_FC2);
        }
    }
    // 4. final LayerNorm on the CLS rows → raw (the /embed body) and L2-normalised copy
    const float *fin = m->cls_only_last ? m->cls_hidden + (int64_t)i0 * H : hidden;
    const bool bf16_rows = fold && !m->cls_only_last;
    hipLaunchKernelGGL(cls_final_kernel<3>, dim3(n), dim3(64), 0, s, fin, bf16_rows ? ln : nullptr,
                       m->cls_only_last ? 1 : T, m->lnf_w, m->lnf_b,
                       c.ln_eps,
                       raw + (int64_t)i0 * H, normed ? normed + (int64_t)i0 * H : nullptr);
    RC_LAUNCH_CHECK();
}

void forward(rc_model *m, const uint8_t *images, int n, int h, int w, float *raw, float *normed, hipStream_t s) {
    const auto &c = m->cfg;
    const int S = c.image_size;
    // 1. preprocess: Pillow-exact resize if needed; rescale/normalize is folded into the
    //    patch GEMM's A loads (a bf16 LUT), so the u8 images are the GEMM's input
    const int tp = m->timers[T_PRE].begin(s);
    const uint8_t *src = resize_batch(m, images, n, h, w, s);
    m->timers[T_PRE].end(tp, s, (h == S && w == S) ? 0.0 : (double)n * (h * w + S * S) * 3);
    // 2-4. encoder: one stream, or P parts of the batch on P streams so that one
    // part's memory-bound kernels (LayerNorm, attention) and GEMM epilogue store
    // bursts overlap another part's MFMA main loops
    int parts = std::max(1, std::min(m->split, kMaxParts));
    while (parts > 1 && n < parts * m->split_min) --parts;
    if (parts == 1) {
        encode(m, src, 0, n, raw, normed, s);
        return;
    }
    RC_HIP(hipEventRecord(m->ev_fork, s));
    for (int p = 1; p < parts; ++p) RC_HIP(hipStreamWaitEvent(m->sp[p], m->ev_fork, 0));
    for (int p = 0; p < parts; ++p) {
        const int i0 = (int)((int64_t)n * p / parts), i1 = (int)((int64_t)n * (p + 1) / parts);
        encode(m, src, i0, i1 - i0, raw, normed, p == 0 ? s : m->sp[p]);
    }
    for (int p = 1; p < parts; ++p) {
        RC_HIP(hipEventRecord(m->ev_join[p], m->sp[p]));
        RC_HIP(hipStreamWaitEvent(s, m->ev_join[p], 0));
    }
}

// One image already at the model's input size: the ~70-kernel chain of forward() captured once
// per buffer triple on a model-owned stream (capture is refused on the legacy default stream, which
// the caller's may be), then replayed on the caller's stream with one hipGraphLaunch — the host
// issues one launch per request instead of ~70 (the reference's /embed is batch 1 by
// construction, embedding/main.py:88-124).  The same kernels and arguments: the same bits.
bool graph_eligible(const rc_model *m, int n, int h, int w) {
    if (!m->use_graphs || n != 1 || h != m->cfg.image_size || w != m->cfg.image_size) return false;
    for (const auto &t : m->timers)
        if (t.enabled) return false;  // event timing needs the stream form
    return true;
}

void forward_graph(rc_model *m, const uint8_t *images, float *raw, float *normed, hipStream_t s) {
    rc_model::EmbedGraph *e = nullptr;
    for (auto &g : m->graphs)
        if (g.images == images && g.raw == raw && g.normed == normed) e = &g;
    if (e == nullptr) {
        const bool repeat = m->last_miss.images == images && m->last_miss.raw == raw && m->last_miss.normed == normed;
        m->last_miss.images = images, m->last_miss.raw = raw, m->last_miss.normed = normed;
        if (m->graph_miss_streak++ >= rc_model::kMaxGraphs && !repeat) {
            // every call brings new buffers: a capture per call would cost more than it saves
            forward(m, images, 1, m->cfg.image_size, m->cfg.image_size, raw, normed, s);
            return;
        }
        if ((int)m->graphs.size() >= rc_model::kMaxGraphs) {
            auto old = std::min_element(m->graphs.begin(), m->graphs.end(),
                                        [](const auto &a, const auto &b) { return a.last < b.last; });
            (void)hipGraphExecDestroy(old->exec);
            m->graphs.erase(old);
        }
        hipStream_t cs = m->sp[1];
        const int S = m->cfg.image_size;
        RC_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
        hipGraph_t g = nullptr;
        try {
            forward(m, images, 1, S, S, raw, normed, cs);
        } catch (...) {
            (void)hipStreamEndCapture(cs, &g);
            if (g) (void)hipGraphDestroy(g);
            throw;
        }
        RC_HIP(hipStreamEndCapture(cs, &g));
        hipGraphExec_t ex = nullptr;
        const hipError_t err = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        RC_HIP(err);
        m->graphs.push_back({images, raw, normed, ex, 0});
        e = &m->graphs.back();
    } else {
        m->graph_miss_streak = 0;
    }
    e->last = ++m->graph_tick;
    RC_HIP(hipGraphLaunch(e->exec, s));
}

}  // namespace

extern "C" {

int rc_model_create(int device, const rc_vit_config *cfg, rc_model **out) {
    return guard([&] {
        RC_REQUIRE(cfg && out, RC_ERR_INVALID, "null argument");
        RC_REQUIRE(cfg->hidden == 768 && cfg->patch == 16 && cfg->heads * 64 == cfg->hidden, RC_ERR_UNSUPPORTED,
                   "this build implements ViT-B/16 geometry (hidden 768, patch 16, head dim 64)");
        RC_REQUIRE(cfg->image_size % cfg->patch == 0 && cfg->image_size <= 224, RC_ERR_UNSUPPORTED,
                   "image_size must be a multiple of 16 and <= 224 (tokens <= 197: attention_v2_kernel's LDS)");
        RC_REQUIRE(cfg->mlp % 256 == 0 && cfg->layers >= 1 && cfg->max_batch >= 1, RC_ERR_INVALID, "bad config");
        DeviceScope ds(device);
        auto *m = new rc_model();
        try {
            m->device = device;
            m->cfg = *cfg;
            m->npatch = (cfg->image_size / cfg->patch) * (cfg->image_size / cfg->patch);
            m->tokens = m->npatch + 1;
            m->kpatch = 3 * cfg->patch * cfg->patch;
            build_shapes(m);
            const int B = cfg->max_batch, H = cfg->hidden;
            // + one tile: the second half of a split batch reads whole tiles past its last row
            m->Mp = round_up(B * m->tokens, gemm_row_pad()) + gemm_row_pad();
            m->hidden = (float *)m->alloc((size_t)m->Mp * H * 4);
            m->ln_stats = (float *)m->alloc((size_t)m->Mp * LN_STRIDE * 4);
            RC_HIP(hipMemset(m->ln_stats, 0, (size_t)m->Mp * LN_STRIDE * 4));  // pad rows: finite scales
            m->ln = (uint16_t *)m->alloc((size_t)m->Mp * H * 2);
            m->qkv = (uint16_t *)m->alloc((size_t)m->Mp * 3 * H * 2);
            m->attn = (uint16_t *)m->alloc((size_t)m->Mp * H * 2);
            m->mlp = (uint16_t *)m->alloc((size_t)m->Mp * cfg->mlp * 2);
            m->resized = (uint8_t *)m->alloc((size_t)B * cfg->image_size * cfg->image_size * 3);
            const int Cp = B + gemm_row_pad();  // compact CLS streams (+ the rows a tile reads past n)
            m->cls_hidden = (float *)m->alloc((size_t)Cp * H * 4);
            m->cls_stats = (float *)m->alloc((size_t)Cp * LN_STRIDE * 4);
            m->cls_part = (float *)m->alloc((size_t)SKINNY_KS * Cp * H * 4);
            RC_HIP(hipMemset(m->cls_stats, 0, (size_t)Cp * LN_STRIDE * 4));
            m->cls_ln = (uint16_t *)m->alloc((size_t)Cp * H * 2);
            m->cls_attn = (uint16_t *)m->alloc((size_t)Cp * H * 2);
            m->cls_mlp = (uint16_t *)m->alloc((size_t)Cp * cfg->mlp * 2);
            RC_HIP(hipMemset(m->cls_hidden, 0, (size_t)Cp * H * 4));
            RC_HIP(hipMemset(m->cls_ln, 0, (size_t)Cp * H * 2));
            RC_HIP(hipMemset(m->cls_attn, 0, (size_t)Cp * H * 2));
            RC_HIP(hipMemset(m->cls_mlp, 0, (size_t)Cp * cfg->mlp * 2));
            // pad rows are read by the GEMM tiles: keep them finite (zero) forever
            RC_HIP(hipMemset(m->hidden, 0, (size_t)m->Mp * H * 4));
            RC_HIP(hipMemset(m->ln, 0, (size_t)m->Mp * H * 2));
            RC_HIP(hipMemset(m->qkv, 0, (size_t)m->Mp * 3 * H * 2));
            RC_HIP(hipMemset(m->attn, 0, (size_t)m->Mp * H * 2));
            RC_HIP(hipMemset(m->mlp, 0, (size_t)m->Mp * cfg->mlp * 2));
            build_lut(m);
            RC_HIP(hipDeviceGetAttribute(&m->ncu, hipDeviceAttributeMultiprocessorCount, device));
            RC_HIP(hipEventCreateWithFlags(&m->ev_fork, hipEventDisableTiming));
            for (int p = 1; p < kMaxParts; ++p) {
                RC_HIP(hipStreamCreateWithFlags(&m->sp[p], hipStreamNonBlocking));
                RC_HIP(hipEventCreateWithFlags(&m->ev_join[p], hipEventDisableTiming));
            }
        } catch (...) {
            delete m;
            throw;
        }
        *out = m;
    });
}

int rc_model_destroy(rc_model *m) {
    return guard([&] {
        if (!m) return;
        DeviceScope ds(m->device);
        delete m;
    });
}

int rc_model_set_weight(rc_model *m, const char *name, const float *host_data, int64_t numel) {
    return guard([&] {
        RC_REQUIRE(m && name && host_data, RC_ERR_INVALID, "null argument");
        std::lock_guard<std::mutex> lk(m->mu);
        m->clear_graphs();
        const std::string key = canonical_name(name);
        auto it = m->shapes.find(key);
        RC_REQUIRE(it != m->shapes.end(), RC_ERR_INVALID, std::string("unknown weight name: ") + name);
        RC_REQUIRE(numel == numel_of(it->second), RC_ERR_INVALID,
                   std::string("size mismatch for ") + name + ": expected " + std::to_string(numel_of(it->second)));
        m->host[key].assign(host_data, host_data + numel);
        m->ready = false;
    });
}

int rc_model_set_preprocess(rc_model *m, int resample, double rescale_factor, const float mean[3], const float std_[3]) {
    return guard([&] {
        RC_REQUIRE(m && mean && std_, RC_ERR_INVALID, "null argument");
        RC_REQUIRE(resample == RC_RESAMPLE_BICUBIC || resample == RC_RESAMPLE_BILINEAR, RC_ERR_UNSUPPORTED,
                   "resample must be BICUBIC (3) or BILINEAR (2)");
        std::lock_guard<std::mutex> lk(m->mu);
        m->clear_graphs();
        DeviceScope ds(m->device);
        const int old_resample = m->resample;
        const double old_rescale = m->rescale;
        float old_mean[3], old_std[3];
        for (int c = 0; c < 3; ++c) {
            old_mean[c] = m->mean[c];
            old_std[c] = m->std_[c];
            m->mean[c] = mean[c];
            m->std_[c] = std_[c];
        }
        m->resample = resample;
        m->rescale = rescale_factor;
        try {
            build_lut(m);
        } catch (...) {  // refused parameters leave the model as it was
            m->resample = old_resample;
            m->rescale = old_rescale;
            for (int c = 0; c < 3; ++c) {
                m->mean[c] = old_mean[c];
                m->std_[c] = old_std[c];
            }
            throw;
        }
    });
}

int rc_model_finalize(rc_model *m) {
    return guard([&] {
        RC_REQUIRE(m, RC_ERR_INVALID, "null model");
        std::lock_guard<std::mutex> lk(m->mu);
        m->clear_graphs();
        DeviceScope ds(m->device);
        for (auto &kv : m->shapes)
            RC_REQUIRE(m->host.count(kv.first), RC_ERR_STATE, "weight not set: " + kv.first);
        auto &h = m->host;
        {   // conv weight [H][3][P][P] → [H][(ky·P + kx)·3 + c]: the implicit GEMM's K order
            const auto &wc = h["embeddings.patch_embeddings.projection.weight"];
            const int P = m->cfg.patch, Hd = m->cfg.hidden;
            std::vector<float> wp(wc.size());
            for (int n = 0; n < Hd; ++n)
                for (int cc = 0; cc < 3; ++cc)
                    for (int ky = 0; ky < P; ++ky)
                        for (int kx = 0; kx < P; ++kx)
                            wp[((size_t)n * P * P + ky * P + kx) * 3 + cc] = wc[(((size_t)n * 3 + cc) * P + ky) * P + kx];
            m->w_patch = upload_bf16(m, {&wp});
        }
        m->b_patch = upload_f32(m, h["embeddings.patch_embeddings.projection.bias"]);
        m->cls = upload_f32(m, h["embeddings.cls_token"]);
        m->pos = upload_f32(m, h["embeddings.position_embeddings"]);
        m->lnf_w = upload_f32(m, h["layernorm.weight"]);
        m->lnf_b = upload_f32(m, h["layernorm.bias"]);
        m->layers.assign(m->cfg.layers, Layer{});
        for (int i = 0; i < m->cfg.layers; ++i) {
            const std::string p = "encoder.layer." + std::to_string(i) + ".";
            Layer &L = m->layers[i];
            L.w_qkv = upload_bf16(m, {&h[p + "attention.attention.query.weight"], &h[p + "attention.attention.key.weight"],
                                      &h[p + "attention.attention.value.weight"]});
            std::vector<float> bqkv;
            for (const char *nm : {"query", "key", "value"}) {
                const auto &b = h[p + "attention.attention." + nm + ".bias"];
                bqkv.insert(bqkv.end(), b.begin(), b.end());
            }
            L.b_qkv = upload_f32(m, bqkv);
            L.w_o = upload_bf16(m, {&h[p + "attention.output.dense.weight"]});
            L.b_o = upload_f32(m, h[p + "attention.output.dense.bias"]);
            L.w_fc1 = upload_bf16(m, {&h[p + "intermediate.dense.weight"]});
            L.b_fc1 = upload_f32(m, h[p + "intermediate.dense.bias"]);
            L.w_fc2 = upload_bf16(m, {&h[p + "output.dense.weight"]});
            L.b_fc2 = upload_f32(m, h[p + "output.dense.bias"]);
            L.ln1_w = upload_f32(m, h[p + "layernorm_before.weight"]);
            L.ln1_b = upload_f32(m, h[p + "layernorm_before.bias"]);
            L.ln2_w = upload_f32(m, h[p + "layernorm_after.weight"]);
            L.ln2_b = upload_f32(m, h[p + "layernorm_after.bias"]);
            std::vector<float> wq;
            for (const char *nm : {"query", "key", "value"}) {
                const auto &w = h[p + "attention.attention." + nm + ".weight"];
                wq.insert(wq.end(), w.begin(), w.end());
            }
            fold_layernorm(m, wq, bqkv, h[p + "layernorm_before.weight"], h[p + "layernorm_before.bias"], &L.w_qkv_f,
                           &L.b_qkv_f, &L.c_qkv);
            fold_layernorm(m, h[p + "intermediate.dense.weight"], h[p + "intermediate.dense.bias"],
                           h[p + "layernorm_after.weight"], h[p + "layernorm_after.bias"], &L.w_fc1_f, &L.b_fc1_f,
                           &L.c_fc1);
        }
        m->host.clear();
        m->ready = true;
    });
}

int rc_embed(rc_model *m, const uint8_t *images, int n, int h, int w, float *raw_out, float *normed_out, void *stream) {
    return guard([&] {
        RC_REQUIRE(m, RC_ERR_INVALID, "null model");
        RC_REQUIRE(n >= 0 && n <= m->cfg.max_batch, RC_ERR_INVALID, "batch size exceeds max_batch");
        RC_REQUIRE(h > 0 && w > 0, RC_ERR_INVALID, "image height/width must be positive");
        if (n == 0) return;
        RC_REQUIRE(images && raw_out, RC_ERR_INVALID, "null buffer");
        std::lock_guard<std::mutex> lk(m->mu);
        RC_REQUIRE(m->ready, RC_ERR_STATE, "model weights not finalized");
        DeviceScope ds(m->device);
        if (graph_eligible(m, n, h, w))
            forward_graph(m, images, raw_out, normed_out, (hipStream_t)stream);
        else
            forward(m, images, n, h, w, raw_out, normed_out, (hipStream_t)stream);
    });
}

int rc_model_set_graphs(rc_model *m, int on) {
    return guard([&] {
        RC_REQUIRE(m, RC_ERR_INVALID, "null model");
        std::lock_guard<std::mutex> lk(m->mu);
        DeviceScope ds(m->device);
        m->clear_graphs();
        m->use_graphs = on != 0;
    });
}

int rc_preprocess(rc_model *m, const uint8_t *images, int n, int h, int w, float *pixel_values, void *stream) {
    return guard([&] {
        RC_REQUIRE(m, RC_ERR_INVALID, "null model");
        RC_REQUIRE(n >= 0 && n <= m->cfg.max_batch && h > 0 && w > 0, RC_ERR_INVALID, "bad batch/shape");
        if (n == 0) return;
        RC_REQUIRE(images && pixel_values, RC_ERR_INVALID, "null buffer");
        std::lock_guard<std::mutex> lk(m->mu);
        DeviceScope ds(m->device);
        hipStream_t s = (hipStream_t)stream;
        const int S = m->cfg.image_size;
        const uint8_t *src = resize_batch(m, images, n, h, w, s);
        hipLaunchKernelGGL(pixel_values_kernel, dim3(grid_for((int64_t)n * 3 * S * S)), dim3(256), 0, s, src, m->lut,
                           pixel_values, n, S);
        RC_LAUNCH_CHECK();
    });
}

int rc_model_timing(rc_model *m, int enable) {
    return guard([&] {
        RC_REQUIRE(m, RC_ERR_INVALID, "null model");
        std::lock_guard<std::mutex> lk(m->mu);
        DeviceScope ds(m->device);
        for (int i = 0; i < T_COUNT; ++i) {
            auto &t = m->timers[i];
            const bool on = (enable >> i) & 1;
            if (on) t.create();
            t.enabled = on;
        }
    });
}

int rc_model_timing_read(rc_model *m, int kernel_id, double *total_ms, int64_t *launches, double *flops) {
    return guard([&] {
        RC_REQUIRE(m, RC_ERR_INVALID, "null model");
        RC_REQUIRE(kernel_id >= 0 && kernel_id < T_COUNT, RC_ERR_INVALID, "bad kernel id");
        std::lock_guard<std::mutex> lk(m->mu);
        DeviceScope ds(m->device);
        auto &t = m->timers[kernel_id];
        t.flush();
        if (total_ms) *total_ms = t.total_ms;
        if (launches) *launches = t.launches;
        if (flops) *flops = t.work;
    });
}

int rc_model_set_parts(rc_model *m, int parts) {
    return guard([&] {
        RC_REQUIRE(m, RC_ERR_INVALID, "null model");
        RC_REQUIRE(parts >= 1 && parts <= kMaxParts, RC_ERR_INVALID, "parts must be in [1, 4]");
        std::lock_guard<std::mutex> lk(m->mu);
        m->clear_graphs();
        m->split = parts;
    });
}

int rc_model_set_ln_fold(rc_model *m, int on) {
    return guard([&] {
        RC_REQUIRE(m, RC_ERR_INVALID, "null model");
        std::lock_guard<std::mutex> lk(m->mu);
        m->clear_graphs();
        m->ln_fold = on != 0;
    });
}

int rc_model_set_last_layer(rc_model *m, int cls_only) {
    return guard([&] {
        RC_REQUIRE(m, RC_ERR_INVALID, "null model");
        std::lock_guard<std::mutex> lk(m->mu);
        m->clear_graphs();
        m->cls_only_last = cls_only != 0;
    });
}

int rc_model_timing_reset(rc_model *m) {
    return guard([&] {
        RC_REQUIRE(m, RC_ERR_INVALID, "null model");
        std::lock_guard<std::mutex> lk(m->mu);
        DeviceScope ds(m->device);
        for (auto &t : m->timers) t.reset();
    });
}

}  // extern "C"

#if defined(RC_GEMM_ABLATION)
// diagnostic builds: device buffer (>= 64 stamps per workgroup of the largest grid) for the
// GEMM kernels' phase stamps, or null to stop stamping
extern "C" int rc_diag_set_stamps(void *dev) {
    return guard([&] { RC_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_rc_stamps), &dev, sizeof(dev))); });
}

// diagnostic builds: the priority of the part streams 1..3 (part 0 runs on the caller's stream):
// -1 = higher than the default, 1 = lower, 0 = default (the product's)
extern "C" int rc_diag_set_part_priority(rc_model *m, int prio) {
    return guard([&] {
        RC_REQUIRE(m && prio >= -1 && prio <= 1, RC_ERR_INVALID, "part priority: -1, 0 or 1");
        std::lock_guard<std::mutex> lk(m->mu);
        DeviceScope ds(m->device);
        m->clear_graphs();
        int lo = 0, hi = 0;
        RC_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
        const int pr = prio < 0 ? hi : (prio > 0 ? lo : 0);
        RC_HIP(hipDeviceSynchronize());
        for (int p = 1; p < kMaxParts; ++p) {
            RC_HIP(hipStreamDestroy(m->sp[p]));
            RC_HIP(hipStreamCreateWithPriority(&m->sp[p], hipStreamNonBlocking, pr));
        }
    });
}

// diagnostic builds: the ping-pong tile order of the wide GEMMs (QKV, fc1): groups of g row tiles
// walked column-major (8, the product's; 0 = row-major)
extern "C" int rc_diag_set_group_m(rc_model *m, int g) {
    return guard([&] {
        RC_REQUIRE(m && g >= 0 && g <= 64, RC_ERR_INVALID, "group_m in [0, 64]");
        std::lock_guard<std::mutex> lk(m->mu);
        m->clear_graphs();
        g_group_m_wide = g;
    });
}

// diagnostic builds: tiles (one wave each) per block of the skinny GEMM (1, the product's; 2; 4)
extern "C" int rc_diag_set_skinny_wpb(rc_model *m, int wpb) {
    return guard([&] {
        RC_REQUIRE(m && (wpb == 1 || wpb == 2 || wpb == 4), RC_ERR_INVALID, "skinny waves per block: 1, 2 or 4");
        std::lock_guard<std::mutex> lk(m->mu);
        m->clear_graphs();
        g_skinny_wpb = wpb;
    });
}

// diagnostic builds: attention_v2_kernel (2, the product's) or attention_v3_kernel (3, lost the
// A/B) for the full-token layers (the same bits)
extern "C" int rc_diag_set_attention(rc_model *m, int form) {
    return guard([&] {
        RC_REQUIRE(m && form >= 2 && form <= 6, RC_ERR_INVALID,
                   "attention form must be 2 (v2), 3 (v3), 4 / 5 (v2 staggered), 6 (v2, default-policy K/V DMA)");
        std::lock_guard<std::mutex> lk(m->mu);
        m->clear_graphs();
        m->attn_form = form;
    });
}

// diagnostic builds: the A/B kernel of the full-batch projections (diag_variant); not in the
// product ABI — the product picks one kernel per shape
extern "C" int rc_diag_set_gemm_variant(rc_model *m, int variant) {
    return guard([&] {
        RC_REQUIRE(m, RC_ERR_INVALID, "null model");
        RC_REQUIRE(variant == GEMM_AUTO || variant == GEMM_PINGPONG || variant == GEMM_W2 || variant == GEMM_PP_IMG ||
                       (variant >= 11 && variant <= 26) || (variant >= 100 && variant < 200),
                   RC_ERR_INVALID, "GEMM variant: 0 auto, 4 ping-pong, 8 two-workgroup, 10 image-aligned, 11-14 producer "
                                   "mixes, 15-17 LN consumers on the two-workgroup kernel, 100 + ABL");
        std::lock_guard<std::mutex> lk(m->mu);
        m->clear_graphs();
        m->gemm_variant = variant;
    });
}
#endif

extern "C" int rc_gemm_bf16(int epi, int variant, const uint16_t *A, const uint16_t *W, const float *bias, int M, int N,
                            int K, void *out, const float *pos, int tokens, void *stream) {
    return guard([&] {
        RC_REQUIRE(A && W && bias && out && M > 0 && N > 0 && K > 0, RC_ERR_INVALID, "bad GEMM arguments");
        GemmArgs a{A, W, bias, M, N, K, (uint16_t *)out, (float *)out, pos, tokens};
        if (variant == GEMM_PP_IMG) {  // image-aligned tiles: `tokens` rows per image (residual epilogue)
#if defined(RC_GEMM_ABLATION)
            RC_REQUIRE(epi == EPI_RESID_F32 && tokens > 0, RC_ERR_INVALID, "variant 10: epi 2 and tokens (rows per image)");
            a.row_step = tokens;
#else
            throw Error(RC_ERR_UNSUPPORTED, "variant 10 (image-aligned tiles) is a diagnostic-build kernel");
#endif
        }
        hipStream_t s = (hipStream_t)stream;
        switch (epi) {
            case EPI_BF16: launch_gemm<EPI_BF16>(a, variant, s); break;
            case EPI_GELU_BF16: launch_gemm<EPI_GELU_BF16>(a, variant, s); break;
            case EPI_RESID_F32: launch_gemm<EPI_RESID_F32>(a, variant, s); break;
            case EPI_PATCH_F32:
                RC_REQUIRE(pos && tokens > 1, RC_ERR_INVALID, "patch epilogue needs pos and tokens");
                launch_gemm<EPI_PATCH_F32>(a, variant, s);
                break;
            default: throw Error(RC_ERR_INVALID, "unknown epilogue");
        }
    });
}
