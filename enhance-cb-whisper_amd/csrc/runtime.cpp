// libcbw native runtime: C ABI (include/cbw.h), parameter loading with
// BatchNorm folding, layer plans and workspace carving for the KWS classifier
// and the Whisper encoder.  No allocation or synchronisation happens in the
// compute entry points (cbw_kws_project / cbw_kws_score / cbw_mel /
// cbw_encoder_hs), so callers can capture them into hipGraphs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "cbw.h"
#include "cbw_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                                   \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) return fail(CBW_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define CHK(expr)                  \
    do {                           \
        int rc_ = (expr);          \
        if (rc_ != CBW_OK) return rc_; \
    } while (0)

int block_zero_page(const void** out);   // a device's 256-byte zero page (defined with the standalone conv entries)

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) { reset(); p = o.p; bytes = o.bytes; o.p = nullptr; o.bytes = 0; }
        return *this;
    }
    ~DevBuf() { reset(); }
    void reset() { if (p) (void)hipFree(p); p = nullptr; bytes = 0; }
    int alloc(size_t n) {
        reset();
        if (hipMalloc(&p, n ? n : 16) != hipSuccess) { p = nullptr; return fail(CBW_ERR_OOM, "hipMalloc failed"); }
        bytes = n;
        return CBW_OK;
    }
    template <class T>
    int upload(const std::vector<T>& v) {
        CHK(alloc(v.size() * sizeof(T)));
        if (hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
            return fail(CBW_ERR_HIP, "hipMemcpy upload failed");
        return CBW_OK;
    }
    template <class T> T* as() const { return (T*)p; }
};

uint16_t f2bf_host(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);   // NaN stays NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

std::vector<uint16_t> to_bf16(const std::vector<float>& v) {
    std::vector<uint16_t> o(v.size());
    for (size_t i = 0; i < v.size(); ++i) o[i] = f2bf_host(v[i]);
    return o;
}

struct ParamStore {
    std::map<std::string, std::vector<float>> host;
    int set(const char* name, const float* data, int64_t numel) {
        if (!name || (!data && numel > 0) || numel < 0) return fail(CBW_ERR_INVALID, "set_param: bad arguments");
        host[name] = std::vector<float>(data, data + numel);
        return CBW_OK;
    }
    const std::vector<float>* get(const std::string& n, size_t numel, int* rc) const {
        auto it = host.find(n);
        if (it == host.end()) { *rc = fail(CBW_ERR_STATE, "missing parameter " + n); return nullptr; }
        if (it->second.size() != numel) {
            *rc = fail(CBW_ERR_INVALID, "parameter " + n + ": expected " + std::to_string(numel) + " elements, got " +
                                            std::to_string(it->second.size()));
            return nullptr;
        }
        *rc = CBW_OK;
        return &it->second;
    }
};

// BatchNorm (eval) folded into a bias-free conv: w' = w * g/sqrt(v+eps), b' = beta - mean * g/sqrt(v+eps)
int fold_bn(const ParamStore& ps, const std::string& bn, int cout, std::vector<float>& scale, std::vector<float>& shift) {
    int rc;
    const auto* g = ps.get(bn + ".weight", cout, &rc); if (!g) return rc;
    const auto* b = ps.get(bn + ".bias", cout, &rc); if (!b) return rc;
    const auto* m = ps.get(bn + ".running_mean", cout, &rc); if (!m) return rc;
    const auto* v = ps.get(bn + ".running_var", cout, &rc); if (!v) return rc;
    scale.resize(cout);
    shift.resize(cout);
    for (int o = 0; o < cout; ++o) {
        const double s = (double)(*g)[o] / std::sqrt((double)(*v)[o] + 1e-5);
        scale[o] = (float)s;
        shift[o] = (float)((double)(*b)[o] - (double)(*m)[o] * s);
    }
    return CBW_OK;
}

struct ConvW {
    DevBuf w, b;
    int cin = 0, cout = 0, k = 1, stride = 1;
    bool relu = false;
};

// torch conv weight [Cout][Cin][k][k] + BN -> f32 [Cout][k][k][Cin] (BN scale folded) + f32 bias
int fold_conv_host(const ParamStore& ps, const std::string& prefix, int cin, int cout, int k, std::vector<float>& o,
                   std::vector<float>& sh) {
    int rc;
    const size_t n = (size_t)cout * cin * k * k;
    const auto* w = ps.get(prefix + ".convolution.weight", n, &rc);
    if (!w) return rc;
    std::vector<float> sc;
    CHK(fold_bn(ps, prefix + ".normalization", cout, sc, sh));
    o.assign(n, 0.f);
    for (int co = 0; co < cout; ++co)
        for (int ci = 0; ci < cin; ++ci)
            for (int kh = 0; kh < k; ++kh)
                for (int kw = 0; kw < k; ++kw)
                    o[(((size_t)co * k + kh) * k + kw) * cin + ci] =
                        (*w)[(((size_t)co * cin + ci) * k + kh) * k + kw] * sc[co];
    return CBW_OK;
}

int load_conv_bn(const ParamStore& ps, const std::string& prefix, ConvW& c) {
    std::vector<float> o, sh;
    CHK(fold_conv_host(ps, prefix, c.cin, c.cout, c.k, o, sh));
    CHK(c.w.upload(to_bf16(o)));
    CHK(c.b.upload(sh));
    return CBW_OK;
}

// expand 1x1 (mid -> cout) and shortcut 1x1 (cin -> cout, stride s) of one bottleneck folded
// into one K-concatenated conv: w [cout][mid + cin], bias = b_expand + b_shortcut.
int load_fused_expand_shortcut(const ParamStore& ps, const std::string& expand, const std::string& shortcut,
                               int mid, int cin, int cout, ConvW& c) {
    std::vector<float> we, be, ws, bs;
    CHK(fold_conv_host(ps, expand, mid, cout, 1, we, be));
    CHK(fold_conv_host(ps, shortcut, cin, cout, 1, ws, bs));
    std::vector<float> w((size_t)cout * (mid + cin)), b(cout);
    for (int co = 0; co < cout; ++co) {
        std::copy(we.begin() + (size_t)co * mid, we.begin() + (size_t)(co + 1) * mid, w.begin() + (size_t)co * (mid + cin));
        std::copy(ws.begin() + (size_t)co * cin, ws.begin() + (size_t)(co + 1) * cin,
                  w.begin() + (size_t)co * (mid + cin) + mid);
        b[co] = be[co] + bs[co];
    }
    CHK(c.w.upload(to_bf16(w)));
    CHK(c.b.upload(b));
    return CBW_OK;
}

// Per-launch HIP-event timing of the implicit-GEMM conv kernels (bench.py roofline):
// events recorded on the launch stream around each conv launch, read after a sync.
struct Prof {
    bool on = false;
    std::vector<hipEvent_t> ev;     // 2 per launch
    std::vector<double> flop;       // algorithmic FLOPs per recorded launch
    std::vector<int> tier;          // 0 the bf16 scoring pass, 1 the compensated re-scoring tier
    std::vector<const char*> kern;  // the kernel each recorded launch ran (cbw_last_conv_kernel: static strings)
    int cur_tier = 0;
    int used = 0;
    ~Prof() { for (auto e : ev) (void)hipEventDestroy(e); }
};

struct Src2 {   // second K-source of a fused 1x1 conv (ConvArgs::x2)
    const void* x;
    int cin, H, W, stride;
};

int launch_conv(const ConvW& c, const void* x, int N, int H, int W, void* y, const void* res, int flags,
                const void* zero, hipStream_t st, int* Ho_out = nullptr, int* Wo_out = nullptr, Prof* prof = nullptr,
                const Src2* src2 = nullptr, float* splitk_ws = nullptr) {
    ConvArgs a{};
    a.x = x; a.w = c.w.p; a.bias = c.b.as<float>(); a.res = res; a.y = y; a.zero = zero;
    if (src2) { a.x2 = src2->x; a.Cin2 = src2->cin; a.H2 = src2->H; a.W2 = src2->W; a.s2 = src2->stride; }
    a.N = N; a.H = H; a.W = W; a.Cin = c.cin; a.Cout = c.cout; a.KH = c.k; a.KW = c.k;
    a.sh = a.sw = c.stride; a.ph = a.pw = c.k / 2;
    a.Ho = (H + 2 * a.ph - a.KH) / a.sh + 1;
    a.Wo = (W + 2 * a.pw - a.KW) / a.sw + 1;
    a.M = N * a.Ho * a.Wo;
    a.res_ld = a.y_ld = c.cout;
    a.flags = flags | (c.relu ? CBW_EPI_RELU : 0);
    if (Ho_out) *Ho_out = a.Ho;
    if (Wo_out) *Wo_out = a.Wo;
    const bool rec = prof && prof->on && (size_t)(2 * prof->used + 1) < prof->ev.size();
    if (rec) HIPCHK(hipEventRecord(prof->ev[2 * prof->used], st));
    cbw_last_conv_kernel = "?";
    if (splitk_ws) HIPCHK(cbw_conv_igemm_splitk(a, cbw_conv_splitk_factor(a), splitk_ws, st));
    else HIPCHK(cbw_conv_igemm(a, st));
    if (rec) {
        HIPCHK(hipEventRecord(prof->ev[2 * prof->used + 1], st));
        prof->flop[prof->used] = 2.0 * a.M * a.Cout * ((double)a.Cin * a.KH * a.KW + (a.x2 ? a.Cin2 : 0));
        prof->tier[prof->used] = prof->cur_tier;
        prof->kern[prof->used] = cbw_last_conv_kernel;
        prof->used++;
    }
    return CBW_OK;
}

size_t align_up(size_t n) { return (n + 255) & ~(size_t)255; }

// ------------------------------------------------------------------ ResNet topology
// HF ResNetConfig defaults as instantiated by efficient_kws/resnet.py:22-38:
// embedding 64, stages [256,512,1024,2048]x[3,4,6,3] bottleneck (resnet-50),
// [64,128,256,512] basic for resnet-18/34; stride 2 in the first layer of stages
// 2-4, in the 3x3 (downsample_in_bottleneck = False); shortcut when shape changes.
struct BlockW {
    ConvW conv[3];
    int nconv = 0;
    bool has_sc = false;
    bool fused_sc = false;   // shortcut folded into conv[2] as a second K-source (bottleneck)
    ConvW sc;
    std::string prefix;      // parameter prefix of the block (bias correction re-folds from it)
    int stage = 0;           // 1..4
};

// e4m3 conv of the fp8 tier (conv_fp8.hip): w [Cout][k][k][Cin] e4m3 = q(w_folded * s_in / alpha), alpha [Cout]
struct ConvF8 {
    DevBuf w, alpha, b;
    int cin = 0, cout = 0, k = 1, stride = 1;
    bool relu = false;
};
struct BlockF8 {
    ConvF8 conv[3];
    bool has_sc = false;
    ConvF8 sc;
    float s_x = 1.f, s_t1 = 1.f, s_t2 = 1.f, s_sc = 1.f;   // activation scales of the block's tensors
    float s_out = 1.f;                                      // the next block's s_x (unused when out_bf16)
    bool out_bf16 = false;                                  // the network's last block: bf16 for the pool / fc
};

// fp32 copies for the exact re-scoring path (kws_exact.hip): BN folded in fp32, no shortcut fusion
struct ConvW32 {
    DevBuf w, b;
    int cin = 0, cout = 0, k = 1, stride = 1;
    bool relu = false;
};
struct BlockW32 {
    ConvW32 conv[3];
    int nconv = 0;
    bool has_sc = false;
    ConvW32 sc;
};

int load_conv_bn32(const ParamStore& ps, const std::string& prefix, ConvW32& c) {
    std::vector<float> o, sh;
    CHK(fold_conv_host(ps, prefix, c.cin, c.cout, c.k, o, sh));
    CHK(c.w.upload(o));
    CHK(c.b.upload(sh));
    return CBW_OK;
}

// compensated bf16 (3-term split) copy of a conv for the middle re-scoring tier: BN folded in fp32, then
// w [Cout][k][k][3 Cin] = [w_hi | w_lo | w_hi] (w_hi = bf16(w), w_lo = bf16(w - w_hi)) against activations
// stored [x_hi | x_lo] (CBW_EPI_SPLIT3) and read as the K-segments [x_hi | x_hi | x_lo] (ConvArgs::xfold),
// so one bf16 MFMA conv over 3 Cin K-channels accumulates x_hi.w_hi + x_hi.w_lo + x_lo.w_hi in fp32 (only
// x_lo.w_lo, ~2^-16 relative, is dropped)
int load_conv_bn_x3(const ParamStore& ps, const std::string& prefix, int cin, int cout, int k, int stride, bool relu,
                    ConvW& c) {
    std::vector<float> o, sh;
    CHK(fold_conv_host(ps, prefix, cin, cout, k, o, sh));
    const size_t taps = (size_t)cout * k * k;
    std::vector<uint16_t> w(taps * 3 * cin);
    for (size_t t = 0; t < taps; ++t)
        for (int ci = 0; ci < cin; ++ci) {
            const float v = o[t * cin + ci];
            const uint16_t hi = f2bf_host(v);
            const uint32_t u = (uint32_t)hi << 16;
            float hv;
            std::memcpy(&hv, &u, 4);
            uint16_t* row = &w[t * 3 * cin];
            row[ci] = hi;
            row[cin + ci] = f2bf_host(v - hv);
            row[2 * cin + ci] = hi;
        }
    c.cin = 3 * cin; c.cout = cout; c.k = k; c.stride = stride; c.relu = relu;
    CHK(c.w.upload(w));
    CHK(c.b.upload(sh));
    return CBW_OK;
}

// one conv of the compensated tier: x bf16 [N][H][W][2C] = [hi | lo] (c.cin = 3C K-channels), y per flags
// (SPLIT3: bf16 [M][2 Cout] [hi | lo] + optional fp32 copy y32; OUT_F32: fp32 [M][Cout]); residual fp32
// [M][Cout] (res_split false) or a [hi | lo] tensor (res_split true)
int launch_conv_x3(const ConvW& c, const void* x, int N, int H, int W, void* y, float* y32, const void* res,
                   bool res_split, int flags, const void* zero, hipStream_t st, int* Ho_out = nullptr,
                   int* Wo_out = nullptr, Prof* prof = nullptr) {
    ConvArgs a{};
    a.x = x; a.w = c.w.p; a.bias = c.b.as<float>(); a.res = res; a.y = y; a.y32 = y32; a.zero = zero;
    a.xfold = c.cin / 3; a.x_ld = 2 * (c.cin / 3);
    a.N = N; a.H = H; a.W = W; a.Cin = c.cin; a.Cout = c.cout; a.KH = a.KW = c.k;
    a.sh = a.sw = c.stride; a.ph = a.pw = c.k / 2;
    a.Ho = (H + 2 * a.ph - a.KH) / a.sh + 1;
    a.Wo = (W + 2 * a.pw - a.KW) / a.sw + 1;
    a.M = N * a.Ho * a.Wo;
    a.res_ld = res_split ? 2 * c.cout : c.cout;
    a.y_ld = (flags & CBW_EPI_SPLIT3) ? 2 * c.cout : c.cout;
    a.flags = flags | (res ? (res_split ? CBW_EPI_RES_SPLIT : CBW_EPI_RES_F32) : 0) | (c.relu ? CBW_EPI_RELU : 0);
    if (Ho_out) *Ho_out = a.Ho;
    if (Wo_out) *Wo_out = a.Wo;
    const bool rec = prof && prof->on && (size_t)(2 * prof->used + 1) < prof->ev.size();
    if (rec) HIPCHK(hipEventRecord(prof->ev[2 * prof->used], st));
    cbw_last_conv_kernel = "?";
    HIPCHK(cbw_conv_igemm(a, st));
    if (rec) {   // the compensated conv's GEMM: K over the three split segments
        HIPCHK(hipEventRecord(prof->ev[2 * prof->used + 1], st));
        prof->flop[prof->used] = 2.0 * a.M * a.Cout * (double)a.Cin * a.KH * a.KW;
        prof->tier[prof->used] = 1;
        prof->kern[prof->used] = cbw_last_conv_kernel;
        prof->used++;
    }
    return CBW_OK;
}

int launch_conv32(const ConvW32& c, const float* x, int N, int H, int W, float* y, const float* res, bool relu,
                  hipStream_t st, int* Ho_out = nullptr, int* Wo_out = nullptr) {
    F32ConvArgs a{};
    a.x = x; a.w = c.w.as<float>(); a.bias = c.b.as<float>(); a.res = res; a.y = y;
    a.N = N; a.H = H; a.W = W; a.Cin = c.cin; a.Cout = c.cout; a.KH = a.KW = c.k;
    a.sh = a.sw = c.stride; a.ph = a.pw = c.k / 2;
    a.Ho = (H + 2 * a.ph - a.KH) / a.sh + 1;
    a.Wo = (W + 2 * a.pw - a.KW) / a.sw + 1;
    a.M = N * a.Ho * a.Wo;
    a.relu = relu ? 1 : 0;
    if (Ho_out) *Ho_out = a.Ho;
    if (Wo_out) *Wo_out = a.Wo;
    HIPCHK(cbw_conv_f32(a, st));
    return CBW_OK;
}

bool sc_fusion_enabled() {   // CBW_NO_SC_FUSION=1 keeps the separate shortcut conv (A/B experiments)
    const char* e = getenv("CBW_NO_SC_FUSION");
    return !(e && atoi(e) != 0);
}

constexpr int KWS_MAX_STREAMS = 4;
// the scoring side streams' priority (CBW_KWS_PRIO, read when the handle creates them; default 0 = normal; -1 = high:
// with the caller's stream also high priority, a normal-priority stream's work -- bench.py's re-scoring tier -- only
// takes the CUs the scoring pass leaves free), clamped to the device's range
hipError_t side_stream_create(hipStream_t* s) {
    const char* e = getenv("CBW_KWS_PRIO");
    int prio = e ? atoi(e) : 0;
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
        prio = std::max(greatest, std::min(least, prio));
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, prio);
}

// keyword chunks round-robin over the caller's stream and kws_streams() - 1 side streams; CBW_KWS_STREAMS=1 runs every
// chunk on the caller's stream (A/B experiments).  3 with 1112-pair chunks (9 per 10k database, 3 per stream) measured
// 6.15-6.16 utt/s vs 6.07-6.10 with 2 x 834 and 5.92-5.96 with 1 (profiles/r06c_chunk_sweep.txt)
int kws_streams() {
    const char* e = getenv("CBW_KWS_STREAMS");
    const int n = e ? atoi(e) : 3;
    return std::max(1, std::min(KWS_MAX_STREAMS, n));
}

// map channels the stem reads: NHWC4 for the efficient_kws classifiers (n_layers <= 4), NHWC16 for
// the original 12-channel CB-Whisper CNN (model/model.py:55-58)
int stem_channels(int n_layers) { return n_layers <= 4 ? 4 : 16; }

bool bottleneck_first_enabled() {   // CBW_NO_BOTTLENECK_FIRST=1 keeps the stage-1 first block on three convs
    const char* e = getenv("CBW_NO_BOTTLENECK_FIRST");
    return !(e && atoi(e));
}
// the last stage-1 block stores the fp8 tier's first tensor in e4m3 itself (default; CBW_FP8_Q8=0: a bf16 tensor and
// the cbw_quant_fp8 pass, bit-identical).  r05b A/B, fp8-first bench at the realistic point: 5.853 vs 5.680 / 5.666
// utt/s, fp8 tier 115.4 vs 119.9 / 121.6 ms per clip, same spotted digest (profiles/r05b_ab.txt)
bool fp8_q8_enabled() {
    const char* e = getenv("CBW_FP8_Q8");
    return !(e && atoi(e) == 0);
}

bool bottleneck_fusion_enabled() {   // CBW_NO_BOTTLENECK_FUSION=1 runs stage-1 blocks as three convs
    const char* e = getenv("CBW_NO_BOTTLENECK_FUSION");
    return !(e && atoi(e) != 0);
}

bool stem_fusion_enabled() {   // CBW_NO_STEM_FUSION=1 runs the separate stem conv + maxpool (A/B experiments)
    const char* e = getenv("CBW_NO_STEM_FUSION");
    return !(e && atoi(e) != 0);
}

}  // namespace

struct cbw_kws {
    cbw_kws_config cfg{};
    ParamStore ps;
    bool finalized = false;
    DevBuf zero;
    DevBuf stem_w, stem_b;
    std::vector<BlockW> blocks;
    int hidden = 2048;
    DevBuf fc_w, fc_b;
    DevBuf fc_b16;   // the bf16 scoring pass's classifier bias: fc_b + the calibrated logit offset (cbw_kws_set_score_offset)
    DevBuf fc_b8;    // the fp8 tier's classifier bias: fc_b + its own logit offset (cbw_kws_set_score_offset_fp8)
    // projector (LE/LEF)
    std::vector<ConvW> p1, p2;
    DevBuf tp_w, tp_b;   // LEF time projector, BN folded: f32 [L][3][U][U] (k, in, out), [L][U]
    Prof prof;
    // fp32 network (exact re-scoring): stem [64][7][7][L], blocks with a separate shortcut, projector
    ConvW32 stem32;
    DevBuf stem16x3_w;   // compensated tier's stem: [64][7][8][16] bf16 = [w_hi | w_lo | w_hi | 0] (3 L <= 16)
    std::vector<BlockW32> blocks32;
    std::vector<BlockW> blocks3;   // compensated bf16 (3-term split) convs of the middle re-scoring tier
    std::vector<ConvW32> p1_32, p2_32;
    // keyword chunks rotate over the caller's stream and these side streams, so one chunk's
    // partially filled launches (tile tails, the short stage-4 convs) and memory-bound layers
    // overlap another chunk's work; fork/join by events, so the whole score call stays
    // capturable into a hipGraph.
    hipStream_t side[KWS_MAX_STREAMS - 1] = {};
    hipEvent_t fork_ev = nullptr, join_ev[KWS_MAX_STREAMS - 1] = {};
    // fp8 first tier (cbw_kws_calibrate_fp8 / cbw_kws_score_fp8): stages 2-4 of ResNet-50 on e4m3 operands,
    // blocks8[i] mirrors blocks[f8_first + i]; the stem and stage 1 run the bf16 network
    std::vector<BlockF8> blocks8;
    int f8_first = -1;
    float f8_in_scale = 1.f;   // scale of the stage-1 output, quantized by cbw_quant_fp8
    // rescore_impl's dispatch throttle: one event per RESCORE_THROTTLE passes, the host waits for the one two back
    hipEvent_t throttle_ev[2] = {};
    ~cbw_kws() {
        for (auto s : side) if (s) (void)hipStreamDestroy(s);
        for (auto e : join_ev) if (e) (void)hipEventDestroy(e);
        if (fork_ev) (void)hipEventDestroy(fork_ev);
        for (auto e : throttle_ev) if (e) (void)hipEventDestroy(e);
    }
};

struct cbw_encoder {
    cbw_encoder_config cfg{};
    ParamStore ps;
    bool finalized = false;
    int cpad = 128;
    DevBuf zero;
    ConvW conv1, conv2;
    DevBuf pos;
    struct Layer {
        DevBuf ln1_g, ln1_b, ln2_g, ln2_b;
        ConvW qkv, out, fc1, fc2;
    };
    std::vector<Layer> layers;
    DevBuf lnf_g, lnf_b;
};

namespace {

int build_resnet(cbw_kws* h) {
    const int L = h->cfg.n_layers;
    std::vector<int> hs, depths;
    bool bottleneck = true;
    switch (h->cfg.resnet_depth) {
        case 50: hs = {256, 512, 1024, 2048}; depths = {3, 4, 6, 3}; break;
        case 34: hs = {64, 128, 256, 512}; depths = {3, 4, 6, 3}; bottleneck = false; break;
        case 18: hs = {64, 128, 256, 512}; depths = {2, 2, 2, 2}; bottleneck = false; break;
        default: return fail(CBW_ERR_INVALID, "resnet_depth must be 18, 34 or 50");
    }
    h->hidden = hs.back();
    const std::string root = "model.feature_extractor";
    // stem: [64][L][7][7] + BN -> bf16 [64][7][8][4]
    {
        int rc;
        const auto* w = h->ps.get(root + ".embedder.embedder.convolution.weight", (size_t)64 * L * 49, &rc);
        if (!w) return rc;
        std::vector<float> sc, sh;
        CHK(fold_bn(h->ps, root + ".embedder.embedder.normalization", 64, sc, sh));
        const int C = stem_channels(L);
        std::vector<float> o((size_t)64 * 7 * 8 * C, 0.f);
        for (int co = 0; co < 64; ++co)
            for (int c = 0; c < L; ++c)
                for (int kh = 0; kh < 7; ++kh)
                    for (int kw = 0; kw < 7; ++kw)
                        o[((co * 7 + kh) * 8 + kw) * C + c] = (*w)[((co * L + c) * 7 + kh) * 7 + kw] * sc[co];
        CHK(h->stem_w.upload(to_bf16(o)));
        CHK(h->stem_b.upload(sh));
    }
    h->blocks.clear();
    int cin = 64;
    for (size_t s = 0; s < hs.size(); ++s) {
        const int cout = hs[s];
        for (int li = 0; li < depths[s]; ++li) {
            const int stride = (li == 0 && s > 0) ? 2 : 1;
            const std::string p = root + ".encoder.stages." + std::to_string(s) + ".layers." + std::to_string(li);
            BlockW b;
            b.prefix = p;
            b.stage = (int)s + 1;
            if (cin != cout || stride != 1) {
                b.has_sc = true;
                b.sc.cin = cin; b.sc.cout = cout; b.sc.k = 1; b.sc.stride = stride; b.sc.relu = false;
                CHK(load_conv_bn(h->ps, p + ".shortcut", b.sc));
            }
            if (bottleneck) {
                const int mid = cout / 4;
                const int ci[3] = {cin, mid, mid}, co[3] = {mid, mid, cout}, k[3] = {1, 3, 1}, st[3] = {1, stride, 1};
                const bool rl[3] = {true, true, false};
                b.nconv = 3;
                for (int j = 0; j < 3; ++j) {
                    b.conv[j].cin = ci[j]; b.conv[j].cout = co[j]; b.conv[j].k = k[j]; b.conv[j].stride = st[j];
                    b.conv[j].relu = rl[j];
                    if (j == 2 && b.has_sc && cout % 128 == 0 && sc_fusion_enabled()) {
                        CHK(load_fused_expand_shortcut(h->ps, p + ".layer.2", p + ".shortcut", mid, cin, cout, b.conv[2]));
                        b.fused_sc = true;
                    } else {
                        CHK(load_conv_bn(h->ps, p + ".layer." + std::to_string(j), b.conv[j]));
                    }
                }
            } else {
                b.nconv = 2;
                b.conv[0].cin = cin; b.conv[0].cout = cout; b.conv[0].k = 3; b.conv[0].stride = stride; b.conv[0].relu = true;
                b.conv[1].cin = cout; b.conv[1].cout = cout; b.conv[1].k = 3; b.conv[1].stride = 1; b.conv[1].relu = false;
                for (int j = 0; j < 2; ++j) CHK(load_conv_bn(h->ps, p + ".layer." + std::to_string(j), b.conv[j]));
            }
            h->blocks.push_back(std::move(b));
            cin = cout;
        }
    }
    int rc;
    const auto* fw = h->ps.get("model.classifier.1.weight", (size_t)2 * h->hidden, &rc);
    if (!fw) return rc;
    const auto* fb = h->ps.get("model.classifier.1.bias", 2, &rc);
    if (!fb) return rc;
    CHK(h->fc_w.upload(*fw));
    CHK(h->fc_b.upload(*fb));
    CHK(h->fc_b16.upload(*fb));
    CHK(h->fc_b8.upload(*fb));
    return CBW_OK;
}

int build_projector(cbw_kws* h) {
    const int L = h->cfg.n_layers, D = h->cfg.embedding_dim, U = h->cfg.proj_units;
    h->p1.clear();
    h->p2.clear();
    h->p1.resize(L);
    h->p2.resize(L);
    for (int l = 0; l < L; ++l) {
        int rc;
        const std::string p = "projector." + std::to_string(l);
        const auto* w1 = h->ps.get(p + ".0.weight", (size_t)(D / 2) * D, &rc); if (!w1) return rc;
        const auto* b1 = h->ps.get(p + ".0.bias", D / 2, &rc); if (!b1) return rc;
        const auto* w2 = h->ps.get(p + ".2.weight", (size_t)U * (D / 2), &rc); if (!w2) return rc;
        const auto* b2 = h->ps.get(p + ".2.bias", U, &rc); if (!b2) return rc;
        h->p1[l].cin = D; h->p1[l].cout = D / 2; h->p1[l].relu = true;
        h->p2[l].cin = D / 2; h->p2[l].cout = U; h->p2[l].relu = false;
        CHK(h->p1[l].w.upload(to_bf16(*w1)));
        CHK(h->p1[l].b.upload(*b1));
        CHK(h->p2[l].w.upload(to_bf16(*w2)));
        CHK(h->p2[l].b.upload(*b2));
    }
    if (h->cfg.variant == 2) {
        std::vector<float> tw((size_t)L * 3 * U * U), tb((size_t)L * U);
        for (int l = 0; l < L; ++l) {
            int rc;
            const std::string p = "time_projector." + std::to_string(l);
            const auto* w = h->ps.get(p + ".0.weight", (size_t)U * U * 3, &rc); if (!w) return rc;
            const auto* b = h->ps.get(p + ".0.bias", U, &rc); if (!b) return rc;
            std::vector<float> sc, sh;
            CHK(fold_bn(h->ps, p + ".1", U, sc, sh));
            for (int o = 0; o < U; ++o) {
                tb[(size_t)l * U + o] = (*b)[o] * sc[o] + sh[o];
                for (int i = 0; i < U; ++i)
                    for (int k = 0; k < 3; ++k)
                        tw[(((size_t)l * 3 + k) * U + i) * U + o] = (*w)[((size_t)o * U + i) * 3 + k] * sc[o];
            }
        }
        CHK(h->tp_w.upload(tw));
        CHK(h->tp_b.upload(tb));
    }
    return CBW_OK;
}

int build_f32(cbw_kws* h) {
    const int L = h->cfg.n_layers;
    std::vector<int> hs, depths;
    bool bottleneck = true;
    switch (h->cfg.resnet_depth) {
        case 50: hs = {256, 512, 1024, 2048}; depths = {3, 4, 6, 3}; break;
        case 34: hs = {64, 128, 256, 512}; depths = {3, 4, 6, 3}; bottleneck = false; break;
        default: hs = {64, 128, 256, 512}; depths = {2, 2, 2, 2}; bottleneck = false; break;
    }
    const std::string root = "model.feature_extractor";
    h->stem32.cin = L; h->stem32.cout = 64; h->stem32.k = 7; h->stem32.stride = 2; h->stem32.relu = true;
    CHK(load_conv_bn32(h->ps, root + ".embedder.embedder", h->stem32));
    if (3 * L <= 16) {   // the compensated stem (cbw_stem16_pool_x3): taps kw padded to 8, channels [hi | lo | hi | 0]
        std::vector<float> o, sh;
        CHK(fold_conv_host(h->ps, root + ".embedder.embedder", L, 64, 7, o, sh));
        std::vector<uint16_t> w16((size_t)64 * 7 * 8 * 16, 0);
        for (int co = 0; co < 64; ++co)
            for (int kh = 0; kh < 7; ++kh)
                for (int kw = 0; kw < 7; ++kw)
                    for (int c = 0; c < L; ++c) {
                        const float v = o[(((size_t)co * 7 + kh) * 7 + kw) * L + c];
                        const uint16_t hi = f2bf_host(v);
                        const uint32_t u = (uint32_t)hi << 16;
                        float hv;
                        std::memcpy(&hv, &u, 4);
                        uint16_t* px = &w16[(((size_t)co * 7 + kh) * 8 + kw) * 16];
                        px[c] = hi;
                        px[L + c] = f2bf_host(v - hv);
                        px[2 * L + c] = hi;
                    }
        CHK(h->stem16x3_w.upload(w16));
    }
    h->blocks32.clear();
    h->blocks3.clear();
    int cin = 64;
    for (size_t s = 0; s < hs.size(); ++s) {
        const int cout = hs[s];
        for (int li = 0; li < depths[s]; ++li) {
            const int stride = (li == 0 && s > 0) ? 2 : 1;
            const std::string p = root + ".encoder.stages." + std::to_string(s) + ".layers." + std::to_string(li);
            BlockW32 b;
            BlockW b3;
            if (cin != cout || stride != 1) {
                b.has_sc = b3.has_sc = true;
                b.sc.cin = cin; b.sc.cout = cout; b.sc.k = 1; b.sc.stride = stride;
                CHK(load_conv_bn32(h->ps, p + ".shortcut", b.sc));
                CHK(load_conv_bn_x3(h->ps, p + ".shortcut", cin, cout, 1, stride, false, b3.sc));
            }
            if (bottleneck) {
                const int mid = cout / 4;
                const int ci[3] = {cin, mid, mid}, co[3] = {mid, mid, cout}, k[3] = {1, 3, 1}, st[3] = {1, stride, 1};
                b.nconv = b3.nconv = 3;
                for (int j = 0; j < 3; ++j) {
                    b.conv[j].cin = ci[j]; b.conv[j].cout = co[j]; b.conv[j].k = k[j]; b.conv[j].stride = st[j];
                    CHK(load_conv_bn32(h->ps, p + ".layer." + std::to_string(j), b.conv[j]));
                    CHK(load_conv_bn_x3(h->ps, p + ".layer." + std::to_string(j), ci[j], co[j], k[j], st[j], true,
                                        b3.conv[j]));
                }
            } else {
                b.nconv = b3.nconv = 2;
                b.conv[0].cin = cin; b.conv[0].cout = cout; b.conv[0].k = 3; b.conv[0].stride = stride;
                b.conv[1].cin = cout; b.conv[1].cout = cout; b.conv[1].k = 3; b.conv[1].stride = 1;
                for (int j = 0; j < 2; ++j) CHK(load_conv_bn32(h->ps, p + ".layer." + std::to_string(j), b.conv[j]));
                CHK(load_conv_bn_x3(h->ps, p + ".layer.0", cin, cout, 3, stride, true, b3.conv[0]));
                CHK(load_conv_bn_x3(h->ps, p + ".layer.1", cout, cout, 3, 1, true, b3.conv[1]));
            }
            h->blocks32.push_back(std::move(b));
            h->blocks3.push_back(std::move(b3));
            cin = cout;
        }
    }
    if (h->cfg.variant > 0) {
        const int D = h->cfg.embedding_dim, U = h->cfg.proj_units;
        h->p1_32.clear();
        h->p2_32.clear();
        h->p1_32.resize(L);
        h->p2_32.resize(L);
        for (int l = 0; l < L; ++l) {
            int rc;
            const std::string p = "projector." + std::to_string(l);
            const auto* w1 = h->ps.get(p + ".0.weight", (size_t)(D / 2) * D, &rc); if (!w1) return rc;
            const auto* b1 = h->ps.get(p + ".0.bias", D / 2, &rc); if (!b1) return rc;
            const auto* w2 = h->ps.get(p + ".2.weight", (size_t)U * (D / 2), &rc); if (!w2) return rc;
            const auto* b2 = h->ps.get(p + ".2.bias", U, &rc); if (!b2) return rc;
            h->p1_32[l].cin = D; h->p1_32[l].cout = D / 2;
            h->p2_32[l].cin = D / 2; h->p2_32[l].cout = U;
            CHK(h->p1_32[l].w.upload(*w1));
            CHK(h->p1_32[l].b.upload(*b1));
            CHK(h->p2_32[l].w.upload(*w2));
            CHK(h->p2_32[l].b.upload(*b2));
        }
    }
    return CBW_OK;
}

// OCP e4m3 (e4m3fn: bias 7, max 448, no infinities) of a float, round to nearest even, saturating
uint8_t f2e4m3_host(float f) {
    const uint8_t sign = std::signbit(f) ? 0x80 : 0;
    float a = std::fabs(f);
    if (std::isnan(a)) return 0x7F;
    if (a >= 448.f) return sign | 0x7E;
    int e;
    const float fr = std::frexp(a, &e);   // a = fr * 2^e, fr in [0.5, 1)
    if (a == 0.f) return sign;
    int E = e - 1;                        // a = 1.m * 2^E
    if (E < -6) {                         // subnormal: multiples of 2^-9
        const float q = std::nearbyint(a * 512.f);   // default rounding mode: to nearest even
        return sign | (uint8_t)q;                    // q == 8 is the smallest normal (exp field 1, mantissa 0)
    }
    float m = std::nearbyint((fr * 2.f - 1.f) * 8.f);
    if (m == 8.f) { m = 0.f; ++E; }
    if (E > 8 || (E == 8 && m == 7.f)) return sign | 0x7E;
    return sign | (uint8_t)(((E + 7) << 3) | (int)m);
}

// a folded conv (torch weight + BN of `prefix`) quantized for the fp8 tier: input tensor scale s_in folded into
// the weights, per-output-channel alpha = max_k |w s_in| / 448
float e4m3_value_host(uint8_t c) {
    const int e = (c >> 3) & 15, m = c & 7;
    const float v = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + (float)m / 8.f, e - 7);
    return (c & 0x80) ? -v : v;
}

// ... with m (the conv input's per-channel means over the calibration pairs, or null) the bias also absorbs the
// mean shift of the rounded weights, sum_{taps, c} m[c] (w - w_e4m3 alpha / s_in) -- the bf16 tier's bias
// correction (apply_bias_correction) for the e4m3 weights
int load_conv_f8(const ParamStore& ps, const std::string& prefix, int cin, int cout, int k, int stride, bool relu,
                 float s_in, ConvF8& c, const double* m = nullptr) {
    std::vector<float> o, sh;
    CHK(fold_conv_host(ps, prefix, cin, cout, k, o, sh));
    const size_t row = (size_t)k * k * cin;
    std::vector<uint8_t> q(o.size());
    std::vector<float> alpha(cout);
    for (int co = 0; co < cout; ++co) {
        float mx = 0.f;
        for (size_t i = 0; i < row; ++i) mx = std::max(mx, std::fabs(o[co * row + i] * s_in));
        const float al = mx > 0.f ? mx / 448.f : 1.f;
        alpha[co] = al;
        double corr = 0.0;
        for (size_t i = 0; i < row; ++i) {
            q[co * row + i] = f2e4m3_host(o[co * row + i] * s_in / al);
            if (m) corr += m[i % cin] * ((double)o[co * row + i] - (double)e4m3_value_host(q[co * row + i]) * al / s_in);
        }
        sh[co] = (float)((double)sh[co] + corr);
    }
    c.cin = cin; c.cout = cout; c.k = k; c.stride = stride; c.relu = relu;
    CHK(c.w.upload(q));
    CHK(c.alpha.upload(alpha));
    CHK(c.b.upload(sh));
    return CBW_OK;
}

int launch_conv_f8(const cbw_kws* h, const ConvF8& c, const uint8_t* x, int N, int H, int W, void* y,
                   const uint8_t* res, float res_scale, bool out_bf16, float y_scale, hipStream_t st, int* Ho_out,
                   int* Wo_out, Prof* prof) {
    F8ConvArgs a{};
    a.x = x; a.w = c.w.as<uint8_t>(); a.alpha = c.alpha.as<float>(); a.bias = c.b.as<float>();
    a.res = res; a.res_scale = res_scale; a.y = y; a.y_inv_scale = 1.f / y_scale; a.out_bf16 = out_bf16 ? 1 : 0;
    a.zero = h->zero.p;
    a.N = N; a.H = H; a.W = W; a.Cin = c.cin; a.Cout = c.cout; a.KH = a.KW = c.k;
    a.sh = a.sw = c.stride; a.ph = a.pw = c.k / 2;
    a.Ho = (H + 2 * a.ph - a.KH) / a.sh + 1;
    a.Wo = (W + 2 * a.pw - a.KW) / a.sw + 1;
    a.M = N * a.Ho * a.Wo;
    a.relu = c.relu ? 1 : 0;
    if (Ho_out) *Ho_out = a.Ho;
    if (Wo_out) *Wo_out = a.Wo;
    if (!cbw_conv_fp8_supported(a)) return fail(CBW_ERR_INVALID, "fp8 conv shape not supported");
    const bool rec = prof && prof->on && (size_t)(2 * prof->used + 1) < prof->ev.size();
    if (rec) HIPCHK(hipEventRecord(prof->ev[2 * prof->used], st));
    cbw_last_conv_kernel = "?";
    HIPCHK(cbw_conv_fp8(a, st));
    if (rec) {
        HIPCHK(hipEventRecord(prof->ev[2 * prof->used + 1], st));
        prof->flop[prof->used] = 2.0 * a.M * a.Cout * (double)a.Cin * a.KH * a.KW;
        prof->tier[prof->used] = prof->cur_tier;
        prof->kern[prof->used] = cbw_last_conv_kernel;
        prof->used++;
    }
    return CBW_OK;
}

// activation sizes of one chunk through the network (elements)
struct KwsPlan {
    size_t maps = 0, big = 0, small = 0;
};

KwsPlan kws_plan(const cbw_kws* h, int Tk, int Tu, int chunk) {
    KwsPlan p;
    const size_t n = (size_t)chunk;
    p.maps = n * Tk * Tu * stem_channels(h->cfg.n_layers);
    int H = (Tk + 6 - 7) / 2 + 1, W = (Tu + 6 - 7) / 2 + 1;
    p.big = n * H * W * 64;
    H = (H + 2 - 3) / 2 + 1;
    W = (W + 2 - 3) / 2 + 1;
    p.big = std::max(p.big, n * H * W * 64);
    for (const auto& b : h->blocks) {
        int Ho = H, Wo = W;
        for (int j = 0; j < b.nconv; ++j) {
            const auto& c = b.conv[j];
            Ho = (Ho + 2 * (c.k / 2) - c.k) / c.stride + 1;
            Wo = (Wo + 2 * (c.k / 2) - c.k) / c.stride + 1;
            const size_t e = n * Ho * Wo * c.cout;
            if (j + 1 < b.nconv) p.small = std::max(p.small, e); else p.big = std::max(p.big, e);
        }
        H = Ho;
        W = Wo;
    }
    return p;
}

}  // namespace

extern "C" {

int cbw_version(void) { return 1; }
const char* cbw_last_error(void) { return g_err.c_str(); }

// ------------------------------------------------------------------ KWS
int cbw_kws_create(const cbw_kws_config* cfg, cbw_kws** out) {
    if (!cfg || !out) return fail(CBW_ERR_INVALID, "null argument");
    if (cfg->n_layers < 1 || cfg->n_layers > 16)
        return fail(CBW_ERR_INVALID, "n_layers must be in [1, 16] (ResNet input channels: NHWC4 or NHWC16 maps)");
    if (cfg->n_layers > 4 && cfg->variant != 0)
        return fail(CBW_ERR_INVALID, "more than 4 layers only without projection (variant 0: the 12-channel CNN)");
    if (cfg->variant < 0 || cfg->variant > 2) return fail(CBW_ERR_INVALID, "variant must be 0 (L), 1 (LE), 2 (LEF)");
    if (cfg->variant > 0 && (cfg->embedding_dim % 128 != 0 || cfg->proj_units != 64))
        return fail(CBW_ERR_INVALID, "LE/LEF need embedding_dim % 128 == 0 and proj_mlp_units == 64");
    if (cfg->variant == 0 && cfg->embedding_dim % 32 != 0)
        return fail(CBW_ERR_INVALID, "L variant needs embedding_dim % 32 == 0");
    auto h = std::make_unique<cbw_kws>();
    h->cfg = *cfg;
    CHK(h->zero.alloc(256));
    HIPCHK(hipMemset(h->zero.p, 0, 256));
    *out = h.release();
    return CBW_OK;
}

int cbw_kws_destroy(cbw_kws* h) {
    delete h;
    return CBW_OK;
}

int cbw_kws_set_param(cbw_kws* h, const char* name, const float* host, int64_t numel) {
    if (!h) return fail(CBW_ERR_INVALID, "null handle");
    h->finalized = false;
    return h->ps.set(name, host, numel);
}

int cbw_kws_finalize(cbw_kws* h) {
    if (!h) return fail(CBW_ERR_INVALID, "null handle");
    CHK(build_resnet(h));
    if (h->cfg.variant > 0) CHK(build_projector(h));
    if (h->cfg.n_layers <= 4) CHK(build_f32(h));
    if (!h->fork_ev) {
        // only the side streams CBW_KWS_STREAMS asks for (more are created on first use, ChunkStreams::begin):
        // a process gets GPU_MAX_HW_QUEUES = 4 hardware queues, and streams beyond that share one in order
        HIPCHK(hipEventCreateWithFlags(&h->fork_ev, hipEventDisableTiming));
        for (int i = 0; i < KWS_MAX_STREAMS - 1; ++i) HIPCHK(hipEventCreateWithFlags(&h->join_ev[i], hipEventDisableTiming));
        const char* all = getenv("CBW_KWS_ALL_SIDE");   // 1: all three side streams up front (the round-1 setup, A/B)
        const int nside = (all && atoi(all) == 1) ? KWS_MAX_STREAMS - 1 : kws_streams() - 1;
        for (int i = 0; i < nside; ++i) HIPCHK(side_stream_create(&h->side[i]));
    }
    h->finalized = true;
    return CBW_OK;
}

int64_t cbw_kws_project_workspace_bytes(cbw_kws* h, int B, int T) {
    if (!h) return -1;
    const int L = h->cfg.n_layers, D = h->cfg.embedding_dim, U = h->cfg.proj_units;
    const size_t rows = (size_t)L * B * T;
    return (int64_t)(align_up(rows * D * 2) + align_up(rows * (D / 2) * 2) + align_up(rows * U * 4));
}

int cbw_kws_project(cbw_kws* h, const float* x, const float* mask, int B, int T, uint16_t* out, float* mask_out,
                    void* ws, int64_t ws_bytes, cbw_stream_t stream) {
    if (!h || !x || !mask || !out || !mask_out) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized) return fail(CBW_ERR_STATE, "cbw_kws_finalize not called");
    if (B <= 0 || T <= 0) return fail(CBW_ERR_INVALID, "B and T must be positive");
    hipStream_t st = (hipStream_t)stream;
    const int L = h->cfg.n_layers, D = h->cfg.embedding_dim, U = h->cfg.proj_units;
    const float eps = 1e-6f;
    if (h->cfg.variant == 0) {
        HIPCHK(cbw_normalize_rows(x, 1, out, 0, 1, B * L, T, D, eps, 0, st));
        HIPCHK(hipMemcpyAsync(mask_out, mask, sizeof(float) * B * L * T, hipMemcpyDeviceToDevice, st));
        return CBW_OK;
    }
    if (ws_bytes < cbw_kws_project_workspace_bytes(h, B, T)) return fail(CBW_ERR_OOM, "projection workspace too small");
    const size_t rows_l = (size_t)B * T;
    char* p = (char*)ws;
    uint16_t* xb = (uint16_t*)p; p += align_up(rows_l * L * D * 2);
    uint16_t* h1 = (uint16_t*)p; p += align_up(rows_l * L * (D / 2) * 2);
    float* h2 = (float*)p;
    HIPCHK(cbw_cast_permute_lbtd(x, xb, B, L, T, D, st));
    for (int l = 0; l < L; ++l) {
        CHK(launch_conv(h->p1[l], xb + (size_t)l * rows_l * D, 1, 1, (int)rows_l, h1 + (size_t)l * rows_l * (D / 2),
                        nullptr, 0, h->zero.p, st));
        CHK(launch_conv(h->p2[l], h1 + (size_t)l * rows_l * (D / 2), 1, 1, (int)rows_l, h2 + (size_t)l * rows_l * U,
                        nullptr, CBW_EPI_OUT_F32, h->zero.p, st));
    }
    if (h->cfg.variant == 1) {
        HIPCHK(cbw_normalize_rows(h2, 1, out, 0, L, B, T, U, eps, 1, st));
        HIPCHK(hipMemcpyAsync(mask_out, mask, sizeof(float) * B * L * T, hipMemcpyDeviceToDevice, st));
    } else {
        HIPCHK(cbw_lef_time_project(h2, h->tp_w.as<float>(), h->tp_b.as<float>(), out, 0, mask, mask_out, L, B, T, U, eps,
                                    st));
    }
    return CBW_OK;
}

}  // extern "C"

namespace {
int64_t chunk_ws_bytes(const cbw_kws* h, int Tk, int Tu, int chunk) {
    const KwsPlan p = kws_plan(h, Tk, Tu, chunk);
    return (int64_t)(align_up(p.maps * 2) + 3 * align_up(p.big * 2) + 2 * align_up(p.small * 2));
}
}  // namespace

extern "C" {

int64_t cbw_kws_workspace_bytes(cbw_kws* h, int Tk, int Tu, int chunk) {
    if (!h || !h->finalized || chunk <= 0) return -1;
    return kws_streams() * chunk_ws_bytes(h, Tk, Tu, chunk);
}

namespace {
// Chunk i runs on stream i % n (0 = caller's stream, then the handle's side streams) with
// workspace slot i % n.  begin(): the side streams wait for work already queued on the caller's
// stream (inputs); end(): the caller's stream waits for every side stream, so completion on the
// caller's stream means every chunk is done.
// With several streams the streaming 1x1 convs (HBM-bound) size their persistent grid for 96 of the 256 CUs, leaving
// the rest to the other streams' MFMA-bound convs (CBW_CS_SHARED_CUS, default 96; 0 = the whole chip): 6.16 vs 6.10
// utt/s in the bench (r06l, profiles/r06l_cs_cus_ab.txt).
int cs_shared_cus() {
    const char* e = getenv("CBW_CS_SHARED_CUS");
    return e ? atoi(e) : 96;
}
struct ChunkStreams {
    cbw_kws* h;
    hipStream_t st;
    int n;
    int saved_cus;
    // the fewest streams that keep the same number of chunk rounds (4 chunks: 2 streams x 2, not 3 streams with one
    // running its second chunk alone; C2's 1000 keywords in chunks of 250)
    static int balanced(int want, int nchunks) {
        const int n = std::max(1, std::min(want, nchunks));
        const int rounds = (nchunks + n - 1) / n;
        return std::max(1, (nchunks + rounds - 1) / rounds);
    }
    ChunkStreams(cbw_kws* h_, hipStream_t st_, int nchunks)
        : h(h_), st(st_), n(h_->fork_ev ? balanced(kws_streams(), nchunks) : 1), saved_cus(cbw_cs_grid_cus) {
        if (n > 1) cbw_cs_grid_cus = cs_shared_cus();
    }
    ~ChunkStreams() { cbw_cs_grid_cus = saved_cus; }
    ChunkStreams(const ChunkStreams&) = delete;
    ChunkStreams& operator=(const ChunkStreams&) = delete;
    int begin() {
        if (n > 1) {
            HIPCHK(hipEventRecord(h->fork_ev, st));
            for (int i = 0; i + 1 < n; ++i) {
                if (!h->side[i]) HIPCHK(side_stream_create(&h->side[i]));
                HIPCHK(hipStreamWaitEvent(h->side[i], h->fork_ev, 0));
            }
        }
        return CBW_OK;
    }
    hipStream_t stream(int i) const { return (i % n) ? h->side[i % n - 1] : st; }
    int slot(int i) const { return i % n; }
    int end() {
        for (int i = 0; i + 1 < n; ++i) {
            HIPCHK(hipEventRecord(h->join_ev[i], h->side[i]));
            HIPCHK(hipStreamWaitEvent(st, h->join_ev[i], 0));
        }
        return CBW_OK;
    }
};

// ResNet over NHWC4 / NHWC16 maps already in `maps` (chunk of kc pairs) -> logits
int resnet_chunk(cbw_kws* h, const KwsPlan& plan, char* ws, int kc, int Tk, int Tu, float* logits, hipStream_t st,
                 bool fp8 = false) {
    char* p = ws + align_up(plan.maps * 2);
    uint16_t* maps = (uint16_t*)ws;
    uint16_t* X = (uint16_t*)p; p += align_up(plan.big * 2);
    uint16_t* Y = (uint16_t*)p; p += align_up(plan.big * 2);
    uint16_t* SC = (uint16_t*)p; p += align_up(plan.big * 2);
    uint16_t* T1 = (uint16_t*)p; p += align_up(plan.small * 2);
    uint16_t* T2 = (uint16_t*)p;
    const int Hs = (Tk + 6 - 7) / 2 + 1, Ws = (Tu + 6 - 7) / 2 + 1;
    const int Hp = (Hs - 1) / 2 + 1, Wp = (Ws - 1) / 2 + 1;
    const int L = h->cfg.n_layers;

    // stem + max-pool of pairs [n0, n0 + nn) into X (every tensor of the chunk is [pair][H][W][C], so a pair range
    // is a contiguous slice of each buffer)
    auto stem = [&](int n0, int nn) -> int {
        uint16_t* xo = X + (size_t)n0 * Hp * Wp * 64;
        const uint16_t* mo = maps + (size_t)n0 * Tk * Tu * stem_channels(L);
        if (stem_channels(L) == 16) {
            HIPCHK(cbw_stem16_pool(mo, h->stem_w.as<uint16_t>(), h->stem_b.as<float>(), xo, nn, Tk, Tu, Hs, Ws, Hp, Wp,
                                   st));
        } else if (stem_fusion_enabled()) {
            HIPCHK(cbw_stem_pool(mo, h->stem_w.as<uint16_t>(), h->stem_b.as<float>(), xo, nn, Tk, Tu, Hs, Ws, Hp, Wp,
                                 st));
        } else {
            uint16_t* yo = Y + (size_t)n0 * Hs * Ws * 64;
            HIPCHK(cbw_stem_conv(mo, h->stem_w.as<uint16_t>(), h->stem_b.as<float>(), yo, nn, Tk, Tu, Hs, Ws, st));
            HIPCHK(cbw_maxpool3s2(yo, xo, nn, Hs, Ws, 64, Hp, Wp, st));
        }
        return CBW_OK;
    };
    // blocks [b0, b1) over pairs [n0, n0 + nn): x / y are the ping-pong buffers' bases, swapped per block
    auto blocks = [&](size_t b0, size_t b1, int n0, int nn, uint16_t*& x, uint16_t*& y, int& H, int& W,
                      int& C) -> int {
        auto at = [&](uint16_t* base, int hh, int ww, int cc) { return base + (size_t)n0 * hh * ww * cc; };
        for (size_t bi = b0; bi < b1; ++bi) {
            const auto& b = h->blocks[bi];
            uint16_t* xo = at(x, H, W, C);
            int Ho = H, Wo = W;
            const void* res = xo;
            const bool s1_first = b.nconv == 3 && b.has_sc && b.fused_sc && b.sc.stride == 1 && b.sc.cin == 64 &&
                                  b.conv[0].cin == 64 && b.conv[0].cout == 64 && b.conv[1].stride == 1 &&
                                  b.conv[2].cout == 256 && bottleneck_fusion_enabled() && bottleneck_first_enabled();
            if (b.has_sc && !b.fused_sc) {
                const int hs = (H - 1) / b.sc.stride + 1, ws2 = (W - 1) / b.sc.stride + 1;
                uint16_t* sco = at(SC, hs, ws2, b.sc.cout);
                CHK(launch_conv(b.sc, xo, nn, H, W, sco, nullptr, 0, h->zero.p, st, nullptr, nullptr, &h->prof));
                res = sco;
            }
            if (s1_first || (b.nconv == 3 && !b.has_sc && b.conv[0].cin == 256 && b.conv[0].cout == 64 &&
                             b.conv[2].cout == 256 && bottleneck_fusion_enabled())) {
                // stage-1 block as one fused kernel (bottleneck.hip): the identity blocks, and the first block with
                // its shortcut folded into the expand
                uint16_t* yo = at(y, H, W, 256);
                const bool rec = h->prof.on && (size_t)(2 * h->prof.used + 1) < h->prof.ev.size();
                if (rec) HIPCHK(hipEventRecord(h->prof.ev[2 * h->prof.used], st));
                if (s1_first)
                    HIPCHK(cbw_bottleneck_s1_first(xo, yo, b.conv[0].w.as<uint16_t>(), b.conv[0].b.as<float>(),
                                                   b.conv[1].w.as<uint16_t>(), b.conv[1].b.as<float>(),
                                                   b.conv[2].w.as<uint16_t>(), b.conv[2].b.as<float>(), h->zero.p, nn,
                                                   H, W, st));
                else
                    HIPCHK(cbw_bottleneck_s1(xo, yo, b.conv[0].w.as<uint16_t>(), b.conv[0].b.as<float>(),
                                             b.conv[1].w.as<uint16_t>(), b.conv[1].b.as<float>(),
                                             b.conv[2].w.as<uint16_t>(), b.conv[2].b.as<float>(), h->zero.p, nn, H, W,
                                             st));
                if (rec) {
                    HIPCHK(hipEventRecord(h->prof.ev[2 * h->prof.used + 1], st));
                    const double cin = s1_first ? 64.0 : 256.0;
                    h->prof.flop[h->prof.used] =
                        2.0 * nn * H * W * (cin * 64 + 64.0 * 576 + 64.0 * 256 + (s1_first ? 64.0 * 256 : 0.0));
                    h->prof.tier[h->prof.used] = h->prof.cur_tier;
                    h->prof.kern[h->prof.used] = s1_first ? "bottleneck_kernel<64>" : "bottleneck_ring_kernel";
                    h->prof.used++;
                }
            } else if (b.nconv == 3) {
                const auto &c0 = b.conv[0], &c1 = b.conv[1], &c2 = b.conv[2];
                const int h1 = (H + 2 * (c0.k / 2) - c0.k) / c0.stride + 1, w1 = (W + 2 * (c0.k / 2) - c0.k) / c0.stride + 1;
                Ho = (h1 + 2 * (c1.k / 2) - c1.k) / c1.stride + 1;
                Wo = (w1 + 2 * (c1.k / 2) - c1.k) / c1.stride + 1;
                uint16_t* t1 = at(T1, h1, w1, c0.cout);
                uint16_t* t2 = at(T2, Ho, Wo, c1.cout);
                uint16_t* yo = at(y, Ho, Wo, c2.cout);
                CHK(launch_conv(c0, xo, nn, H, W, t1, nullptr, 0, h->zero.p, st, nullptr, nullptr, &h->prof));
                CHK(launch_conv(c1, t1, nn, h1, w1, t2, nullptr, 0, h->zero.p, st, nullptr, nullptr, &h->prof));
                if (b.fused_sc) {   // y = relu([T2 | x strided] . [W_expand ; W_shortcut] + b): no shortcut tensor
                    const Src2 s2{xo, b.sc.cin, H, W, b.sc.stride};
                    CHK(launch_conv(c2, t2, nn, Ho, Wo, yo, nullptr, CBW_EPI_RELU, h->zero.p, st, nullptr, nullptr,
                                    &h->prof, &s2));
                } else {
                    CHK(launch_conv(c2, t2, nn, Ho, Wo, yo, res, CBW_EPI_RELU, h->zero.p, st, nullptr, nullptr,
                                    &h->prof));
                }
            } else {
                const auto &c0 = b.conv[0], &c1 = b.conv[1];
                Ho = (H + 2 * (c0.k / 2) - c0.k) / c0.stride + 1;
                Wo = (W + 2 * (c0.k / 2) - c0.k) / c0.stride + 1;
                uint16_t* t1 = at(T1, Ho, Wo, c0.cout);
                uint16_t* yo = at(y, Ho, Wo, c1.cout);
                CHK(launch_conv(c0, xo, nn, H, W, t1, nullptr, 0, h->zero.p, st, nullptr, nullptr, &h->prof));
                CHK(launch_conv(c1, t1, nn, Ho, Wo, yo, res, CBW_EPI_RELU, h->zero.p, st, nullptr, nullptr, &h->prof));
            }
            std::swap(x, y);
            H = Ho;
            W = Wo;
            C = b.conv[b.nconv - 1].cout;
        }
        return CBW_OK;
    };

    if (fp8) {   // the fp8 tier: stem + stage 1 in bf16, then the e4m3 blocks (conv_fp8.hip)
        int H = Hp, W = Wp, C = 64;
        uint16_t *x = X, *y = Y;
        CHK(stem(0, kc));
        // the last stage-1 block stores its output in e4m3 when it runs fused (bottleneck.hip, Q8; CBW_FP8_Q8=0 off):
        // no separate quantization pass; otherwise the bf16 output is quantized by cbw_quant_fp8 (same values)
        if (h->f8_first < 1) return fail(CBW_ERR_STATE, "fp8 tier: no bf16 stage before the e4m3 blocks");
        const size_t lb = (size_t)h->f8_first - 1;
        const auto& b1 = h->blocks[lb];
        const bool q8 = fp8_q8_enabled() && b1.nconv == 3 && !b1.has_sc && b1.conv[0].cin == 256 &&
                        b1.conv[0].cout == 64 && b1.conv[2].cout == 256 && bottleneck_fusion_enabled();
        CHK(blocks(0, q8 ? lb : (size_t)h->f8_first, 0, kc, x, y, H, W, C));
        uint8_t* cur = (uint8_t*)y;
        uint8_t* other = (uint8_t*)x;
        if (q8) {
            // the same per-launch event / FLOP / tier record blocks() makes for every fused stage-1 block
            const bool rec = h->prof.on && (size_t)(2 * h->prof.used + 1) < h->prof.ev.size();
            if (rec) HIPCHK(hipEventRecord(h->prof.ev[2 * h->prof.used], st));
            HIPCHK(cbw_bottleneck_s1_q8(x, cur, b1.conv[0].w.as<uint16_t>(), b1.conv[0].b.as<float>(),
                                        b1.conv[1].w.as<uint16_t>(), b1.conv[1].b.as<float>(), b1.conv[2].w.as<uint16_t>(),
                                        b1.conv[2].b.as<float>(), 1.f / h->f8_in_scale, kc, H, W, st));
            if (rec) {
                HIPCHK(hipEventRecord(h->prof.ev[2 * h->prof.used + 1], st));
                h->prof.flop[h->prof.used] = 2.0 * kc * H * W * (256.0 * 64 + 64.0 * 576 + 64.0 * 256);
                h->prof.tier[h->prof.used] = h->prof.cur_tier;
                h->prof.kern[h->prof.used] = "bottleneck_ring_kernel (e4m3 out)";
                h->prof.used++;
            }
            C = 256;
        } else {
            HIPCHK(cbw_quant_fp8(x, cur, (int64_t)kc * H * W * C, 1.f / h->f8_in_scale, st));
        }
        uint8_t* sc8 = (uint8_t*)SC;
        uint8_t* t1 = (uint8_t*)T1;
        uint8_t* t2 = (uint8_t*)T2;
        for (const BlockF8& b : h->blocks8) {
            const uint8_t* res = cur;
            float rs = b.s_x;
            if (b.has_sc) {
                CHK(launch_conv_f8(h, b.sc, cur, kc, H, W, sc8, nullptr, 0.f, false, b.s_sc, st, nullptr, nullptr,
                                   &h->prof));
                res = sc8;
                rs = b.s_sc;
            }
            int h1, w1, Ho, Wo;
            CHK(launch_conv_f8(h, b.conv[0], cur, kc, H, W, t1, nullptr, 0.f, false, b.s_t1, st, &h1, &w1, &h->prof));
            CHK(launch_conv_f8(h, b.conv[1], t1, kc, h1, w1, t2, nullptr, 0.f, false, b.s_t2, st, &Ho, &Wo, &h->prof));
            CHK(launch_conv_f8(h, b.conv[2], t2, kc, Ho, Wo, other, res, rs, b.out_bf16, b.s_out, st, nullptr, nullptr,
                               &h->prof));
            std::swap(cur, other);
            H = Ho;
            W = Wo;
            C = b.conv[2].cout;
        }
        HIPCHK(cbw_pool_fc((const uint16_t*)cur, h->fc_w.as<float>(), h->fc_b8.as<float>(), logits, kc, H * W, C, st));
        return CBW_OK;
    }
    int H = Hp, W = Wp, C = 64;
    uint16_t *x = X, *y = Y;
    CHK(stem(0, kc));
    CHK(blocks(0, h->blocks.size(), 0, kc, x, y, H, W, C));
    HIPCHK(cbw_pool_fc(x, h->fc_w.as<float>(), h->fc_b16.as<float>(), logits, kc, H * W, C, st));
    return CBW_OK;
}
}  // namespace

int cbw_kws_score(cbw_kws* h, const uint16_t* utt, const float* utt_mask, const uint16_t* kwd, const float* kwd_mask,
                  int K, int Tk, int Tu, float* logits, float* features, int chunk, void* ws, int64_t ws_bytes,
                  cbw_stream_t stream) {
    if (!h || !utt || !utt_mask || (K > 0 && (!kwd || !kwd_mask || !logits))) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized) return fail(CBW_ERR_STATE, "cbw_kws_finalize not called");
    if (K == 0) return CBW_OK;
    if (K < 0 || Tk < 7 || Tu < 7 || chunk <= 0) return fail(CBW_ERR_INVALID, "bad K/Tk/Tu/chunk");
    if (ws_bytes < cbw_kws_workspace_bytes(h, Tk, Tu, chunk)) return fail(CBW_ERR_OOM, "score workspace too small");
    hipStream_t st = (hipStream_t)stream;
    const int L = h->cfg.n_layers;
    const int E = h->cfg.variant == 0 ? h->cfg.embedding_dim : h->cfg.proj_units;
    const KwsPlan plan = kws_plan(h, Tk, Tu, chunk);
    const int64_t per = chunk_ws_bytes(h, Tk, Tu, chunk);
    ChunkStreams cs(h, st, (K + chunk - 1) / chunk);
    CHK(cs.begin());
    for (int k0 = 0, i = 0; k0 < K; k0 += chunk, ++i) {
        const int kc = std::min(chunk, K - k0);
        hipStream_t s = cs.stream(i);
        char* w = (char*)ws + cs.slot(i) * per;
        uint16_t* maps = (uint16_t*)w;
        const uint16_t* kc_kwd = kwd + (size_t)k0 * L * Tk * E;
        const float* kc_mask = kwd_mask + (size_t)k0 * L * Tk;
        HIPCHK(cbw_sim_maps(kc_kwd, kc_mask, utt, utt_mask, maps, kc, L, Tk, Tu, E, s));
        if (features) HIPCHK(cbw_sim_to_nchw(maps, features + (size_t)k0 * L * Tk * Tu, kc, L, Tk, Tu, s));
        CHK(resnet_chunk(h, plan, w, kc, Tk, Tu, logits + (size_t)k0 * 2, s));
    }
    return cs.end();
}

int cbw_kws_score_fp8(cbw_kws* h, const uint16_t* utt, const float* utt_mask, const uint16_t* kwd,
                      const float* kwd_mask, int K, int Tk, int Tu, float* logits, int chunk, void* ws, int64_t ws_bytes,
                      cbw_stream_t stream) {
    if (!h || !utt || !utt_mask || (K > 0 && (!kwd || !kwd_mask || !logits))) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized) return fail(CBW_ERR_STATE, "cbw_kws_finalize not called");
    if (h->blocks8.empty() || h->f8_first < 0) return fail(CBW_ERR_STATE, "fp8 tier not calibrated (cbw_kws_calibrate_fp8)");
    if (K == 0) return CBW_OK;
    if (K < 0 || Tk < 7 || Tu < 7 || chunk <= 0) return fail(CBW_ERR_INVALID, "bad K/Tk/Tu/chunk");
    if (ws_bytes < cbw_kws_workspace_bytes(h, Tk, Tu, chunk)) return fail(CBW_ERR_OOM, "score workspace too small");
    hipStream_t st = (hipStream_t)stream;
    const int L = h->cfg.n_layers;
    const int E = h->cfg.variant == 0 ? h->cfg.embedding_dim : h->cfg.proj_units;
    const KwsPlan plan = kws_plan(h, Tk, Tu, chunk);
    const int64_t per = chunk_ws_bytes(h, Tk, Tu, chunk);
    ChunkStreams cs(h, st, (K + chunk - 1) / chunk);
    CHK(cs.begin());
    const int tier0 = h->prof.cur_tier;
    h->prof.cur_tier = 2;
    int rc = CBW_OK;
    for (int k0 = 0, i = 0; k0 < K && rc == CBW_OK; k0 += chunk, ++i) {
        const int kc = std::min(chunk, K - k0);
        hipStream_t s = cs.stream(i);
        char* w = (char*)ws + cs.slot(i) * per;
        const hipError_t e = cbw_sim_maps(kwd + (size_t)k0 * L * Tk * E, kwd_mask + (size_t)k0 * L * Tk, utt, utt_mask,
                                          (uint16_t*)w, kc, L, Tk, Tu, E, s);
        if (e != hipSuccess) { rc = fail(CBW_ERR_HIP, hipGetErrorString(e)); break; }
        rc = resnet_chunk(h, plan, w, kc, Tk, Tu, logits + (size_t)k0 * 2, s, true);
    }
    h->prof.cur_tier = tier0;
    CHK(rc);
    return cs.end();
}

int cbw_kws_set_score_offset_fp8(cbw_kws* h, const float* offset) {
    if (!h || !offset) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized || h->fc_b8.bytes != 2 * sizeof(float)) return fail(CBW_ERR_STATE, "cbw_kws_finalize not called");
    int rc;
    const auto* fb = h->ps.get("model.classifier.1.bias", 2, &rc);
    if (!fb) return rc;
    const float b[2] = {(*fb)[0] + offset[0], (*fb)[1] + offset[1]};
    // the bias is read by scoring launches on any stream: drain the device before overwriting it in place
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(h->fc_b8.p, b, sizeof(b), hipMemcpyHostToDevice));
    return CBW_OK;
}

int cbw_kws_fp8_scales(cbw_kws* h, float* scales, int max_n) {
    if (!h || (max_n > 0 && !scales)) return fail(CBW_ERR_INVALID, "null argument");
    const int n = (int)h->blocks8.size() * 4 + 1;
    if (max_n >= 1) scales[0] = h->f8_in_scale;
    for (size_t i = 0; i < h->blocks8.size(); ++i) {
        const BlockF8& b = h->blocks8[i];
        const float v[4] = {b.s_x, b.s_t1, b.s_t2, b.has_sc ? b.s_sc : 0.f};
        for (int j = 0; j < 4; ++j)
            if ((int)(1 + 4 * i + j) < max_n) scales[1 + 4 * i + j] = v[j];
    }
    return n;
}

int cbw_conv2d_fp8(const uint8_t* x, const uint8_t* w, const float* alpha, const float* bias, const uint8_t* res,
                   float res_scale, void* y, float y_scale, int out_bf16, int relu, int N, int H, int W, int Cin,
                   int Cout, int k, int stride, cbw_stream_t stream) {
    const void* zp = nullptr;
    CHK(block_zero_page(&zp));
    F8ConvArgs a{};
    a.x = x; a.w = w; a.alpha = alpha; a.bias = bias; a.res = res; a.res_scale = res_scale; a.y = y;
    a.y_inv_scale = 1.f / y_scale; a.out_bf16 = out_bf16; a.zero = zp; a.relu = relu;
    a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.KH = a.KW = k; a.sh = a.sw = stride;
    a.ph = a.pw = k / 2;
    a.Ho = (H + 2 * a.ph - k) / stride + 1;
    a.Wo = (W + 2 * a.pw - k) / stride + 1;
    a.M = N * a.Ho * a.Wo;
    if (!cbw_conv_fp8_supported(a) || y_scale <= 0.f)
        return fail(CBW_ERR_INVALID, "cbw_conv2d_fp8: 1x1 / 3x3, Cin % 128 == 0, Cout % 128 == 0, positive scales");
    HIPCHK(cbw_conv_fp8(a, (hipStream_t)stream));
    return CBW_OK;
}

int cbw_fp8_probe(int what, const void* a, const void* b, void* out, void* out2, int n, cbw_stream_t stream) {
    hipStream_t st = (hipStream_t)stream;
    if (what >= 0 && what <= 3) {   // the MFMA operand map: a = A [16][128] e4m3, b = B^T [16][128], out = C f32 [16][16]
        HIPCHK(cbw_mfma_fp8_probe((const uint8_t*)a, (const uint8_t*)b, (float*)out, what, st));
        return CBW_OK;
    }
    if (what == 4) {   // conversions: a = f32 [n] -> out = e4m3 [n] (saturating), out2 = f32 [n] decoded
        HIPCHK(cbw_cvt_fp8_probe((const float*)a, (uint8_t*)out, (float*)out2, n, st));
        return CBW_OK;
    }
    return fail(CBW_ERR_INVALID, "cbw_fp8_probe: what in 0..4");
}

int cbw_kws_classify(cbw_kws* h, const float* maps_nchw, int K, int Tk, int Tu, float* logits, int chunk, void* ws,
                     int64_t ws_bytes, cbw_stream_t stream) {
    if (!h || (K > 0 && (!maps_nchw || !logits))) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized) return fail(CBW_ERR_STATE, "cbw_kws_finalize not called");
    if (K == 0) return CBW_OK;
    if (K < 0 || Tk < 7 || Tu < 7 || chunk <= 0) return fail(CBW_ERR_INVALID, "bad K/Tk/Tu/chunk");
    if (ws_bytes < cbw_kws_workspace_bytes(h, Tk, Tu, chunk)) return fail(CBW_ERR_OOM, "score workspace too small");
    hipStream_t st = (hipStream_t)stream;
    const int L = h->cfg.n_layers;
    const KwsPlan plan = kws_plan(h, Tk, Tu, chunk);
    const int64_t per = chunk_ws_bytes(h, Tk, Tu, chunk);
    ChunkStreams cs(h, st, (K + chunk - 1) / chunk);
    CHK(cs.begin());
    for (int k0 = 0, i = 0; k0 < K; k0 += chunk, ++i) {
        const int kc = std::min(chunk, K - k0);
        hipStream_t s = cs.stream(i);
        char* w = (char*)ws + cs.slot(i) * per;
        if (stem_channels(L) == 16)
            HIPCHK(cbw_nchw_to_nhwc16(maps_nchw + (size_t)k0 * L * Tk * Tu, (uint16_t*)w, kc, L, Tk, Tu, s));
        else
            HIPCHK(cbw_nchw_to_nhwc4(maps_nchw + (size_t)k0 * L * Tk * Tu, (uint16_t*)w, kc, L, Tk, Tu, s));
        CHK(resnet_chunk(h, plan, w, kc, Tk, Tu, logits + (size_t)k0 * 2, s));
    }
    return cs.end();
}

// ---- CB-Whisper original spotter (cb_whisper.py:93-129, :189-210)
namespace {
struct ResizedWs {
    int TuP = 0;
    int64_t rmax = 0, utt_bytes = 0, sim_bytes = 0, chunk_bytes = 0;
};
int resized_ws(const cbw_kws* h, const int32_t* off_host, int K, int Tu, int D, int Ho, int Wo, int chunk,
               ResizedWs& r) {
    if (!off_host || K < 0 || Tu <= 0 || D <= 0 || Ho < 7 || Wo < 7 || chunk <= 0)
        return fail(CBW_ERR_INVALID, "bad arguments");
    const int L = h->cfg.n_layers;
    r.TuP = (Tu + 127) / 128 * 128;
    r.rmax = 0;
    for (int k0 = 0; k0 < K; k0 += chunk) {
        const int kc = std::min(chunk, K - k0);
        const int64_t rows = (int64_t)off_host[k0 + kc] - off_host[k0];
        for (int k = k0; k < k0 + kc; ++k)
            if (off_host[k + 1] <= off_host[k]) return fail(CBW_ERR_INVALID, "every keyword needs >= 1 frame");
        r.rmax = std::max(r.rmax, rows);
    }
    r.utt_bytes = (int64_t)align_up((size_t)L * r.TuP * D * 2);
    r.sim_bytes = (int64_t)align_up((size_t)L * std::max<int64_t>(r.rmax, 1) * r.TuP * 4);
    r.chunk_bytes = chunk_ws_bytes(h, Ho, Wo, chunk);
    return CBW_OK;
}
}  // namespace

int64_t cbw_kws_score_resized_workspace_bytes(cbw_kws* h, const int32_t* off_host, int K, int Tu, int D, int Ho,
                                              int Wo, int chunk) {
    if (!h || !h->finalized) return -1;
    ResizedWs r;
    if (resized_ws(h, off_host, K, Tu, D, Ho, Wo, chunk, r) != CBW_OK) return -1;
    return r.utt_bytes + r.sim_bytes + r.chunk_bytes;
}

int cbw_kws_score_resized(cbw_kws* h, const uint16_t* utt, int Tu, const uint16_t* kwd, int R, int D,
                          const int32_t* off_dev, const int32_t* off_host, int K, int Ho, int Wo, float* logits,
                          int chunk, void* ws, int64_t ws_bytes, cbw_stream_t stream) {
    if (!h || !utt || (K > 0 && (!kwd || !off_dev || !off_host || !logits))) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized) return fail(CBW_ERR_STATE, "cbw_kws_finalize not called");
    if (h->cfg.variant != 0) return fail(CBW_ERR_INVALID, "the resized-similarity path takes raw hs (variant 0)");
    if (K == 0) return CBW_OK;
    if (D % 64) return fail(CBW_ERR_INVALID, "D must be a multiple of 64");
    ResizedWs r;
    CHK(resized_ws(h, off_host, K, Tu, D, Ho, Wo, chunk, r));
    if (off_host[0] < 0 || off_host[K] > R) return fail(CBW_ERR_INVALID, "keyword rows out of range");
    if (ws_bytes < r.utt_bytes + r.sim_bytes + r.chunk_bytes) return fail(CBW_ERR_OOM, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    const int L = h->cfg.n_layers;
    char* p = (char*)ws;
    uint16_t* uttP = (uint16_t*)p; p += r.utt_bytes;
    float* sims = (float*)p; p += r.sim_bytes;
    char* cws = p;
    // utterance rows zero-padded to a multiple of 128: they are the GEMM's output channels
    HIPCHK(hipMemsetAsync(uttP, 0, r.utt_bytes, st));
    HIPCHK(hipMemcpy2DAsync(uttP, (size_t)r.TuP * D * 2, utt, (size_t)Tu * D * 2, (size_t)Tu * D * 2, L,
                            hipMemcpyDeviceToDevice, st));
    const KwsPlan plan = kws_plan(h, Ho, Wo, chunk);
    for (int k0 = 0; k0 < K; k0 += chunk) {
        const int kc = std::min(chunk, K - k0);
        const int rows = off_host[k0 + kc] - off_host[k0];
        for (int l = 0; l < L; ++l) {   // sim[l] = kwd[l] . utt[l]^T  (cb_whisper.py:196, inputs normalised)
            ConvArgs a{};
            a.x = kwd + ((size_t)l * R + off_host[k0]) * D;
            a.w = uttP + (size_t)l * r.TuP * D;
            a.y = sims + (size_t)l * r.rmax * r.TuP;
            a.zero = h->zero.p;
            a.N = 1; a.H = 1; a.W = rows; a.Cin = D; a.Ho = 1; a.Wo = rows; a.Cout = r.TuP; a.KH = a.KW = 1;
            a.sh = a.sw = 1; a.M = rows; a.res_ld = a.y_ld = r.TuP; a.flags = CBW_EPI_OUT_F32;
            HIPCHK(cbw_conv_igemm(a, st));
        }
        HIPCHK(cbw_sim_resize(sims, r.rmax * r.TuP, r.TuP, off_dev, k0, kc, L, Tu, Ho, Wo, (uint16_t*)cws, st));
        CHK(resnet_chunk(h, plan, cws, kc, Ho, Wo, logits + (size_t)k0 * 2, st));
    }
    return CBW_OK;
}

int cbw_kws_profile(cbw_kws* h, int max_launches) {
    if (!h || max_launches < 0) return fail(CBW_ERR_INVALID, "bad arguments");
    for (auto e : h->prof.ev) (void)hipEventDestroy(e);
    h->prof.ev.clear();
    h->prof.flop.assign(max_launches, 0.0);
    h->prof.tier.assign(max_launches, 0);
    h->prof.kern.assign(max_launches, "");
    h->prof.cur_tier = 0;
    h->prof.used = 0;
    h->prof.on = max_launches > 0;
    for (int i = 0; i < 2 * max_launches; ++i) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        h->prof.ev.push_back(e);
    }
    return CBW_OK;
}

int cbw_kws_profile_records(cbw_kws* h, double* start_ms, double* end_ms, double* flop, int max_records) {
    if (!h || max_records < 0 || (max_records > 0 && (!start_ms || !end_ms || !flop)))
        return fail(CBW_ERR_INVALID, "bad arguments");
    const int n = std::min(max_records, h->prof.used);
    for (int i = 0; i < n; ++i) {
        float a = 0.f, b = 0.f;
        HIPCHK(hipEventSynchronize(h->prof.ev[2 * i + 1]));
        HIPCHK(hipEventElapsedTime(&a, h->prof.ev[0], h->prof.ev[2 * i]));
        HIPCHK(hipEventElapsedTime(&b, h->prof.ev[0], h->prof.ev[2 * i + 1]));
        start_ms[i] = a;
        end_ms[i] = b;
        flop[i] = h->prof.flop[i];
    }
    return h->prof.used;
}

int cbw_kws_profile_tiers(cbw_kws* h, int32_t* tier, int max_records) {
    if (!h || max_records < 0 || (max_records > 0 && !tier)) return fail(CBW_ERR_INVALID, "bad arguments");
    const int n = std::min(max_records, h->prof.used);
    for (int i = 0; i < n; ++i) tier[i] = h->prof.tier[i];
    return h->prof.used;
}

int cbw_kws_profile_kernels(cbw_kws* h, const char** kernel, int max_records) {
    if (!h || max_records < 0 || (max_records > 0 && !kernel)) return fail(CBW_ERR_INVALID, "bad arguments");
    const int n = std::min(max_records, h->prof.used);
    for (int i = 0; i < n; ++i) kernel[i] = h->prof.kern[i];
    return h->prof.used;
}

int cbw_kws_profile_read(cbw_kws* h, double* ms, double* flop, int* n) {
    if (!h || !ms || !flop || !n) return fail(CBW_ERR_INVALID, "bad arguments");
    // busy time of the conv family = union of the launch intervals (chunks on two streams overlap)
    double f = 0.0;
    std::vector<std::pair<double, double>> iv;
    for (int i = 0; i < h->prof.used; ++i) {
        float a = 0.f, b = 0.f;
        HIPCHK(hipEventSynchronize(h->prof.ev[2 * i + 1]));
        HIPCHK(hipEventElapsedTime(&a, h->prof.ev[0], h->prof.ev[2 * i]));
        HIPCHK(hipEventElapsedTime(&b, h->prof.ev[0], h->prof.ev[2 * i + 1]));
        iv.emplace_back(a, b);
        f += h->prof.flop[i];
    }
    std::sort(iv.begin(), iv.end());
    double t = 0.0, cs = -1e300, ce = -1e300;
    for (const auto& p : iv) {
        if (p.first > ce) {
            if (ce > cs) t += ce - cs;
            cs = p.first;
            ce = p.second;
        } else {
            ce = std::max(ce, p.second);
        }
    }
    if (ce > cs) t += ce - cs;
    *ms = t;
    *flop = f;
    *n = h->prof.used;
    h->prof.used = 0;
    return CBW_OK;
}

// ------------------------------------------------------------------ fp32 re-scoring (kws_exact.hip)
namespace {
constexpr int EXACT_CHUNK = 32;
constexpr int RESCORE_THROTTLE = 8;   // passes per throttle event in rescore_impl (<= 16 passes, ~1 000 dispatches)

struct ExactPlan {
    size_t maps = 0, stem = 0, big = 0, small = 0;
};

extern "C++" ExactPlan exact_plan(const cbw_kws* h, int Tk, int Tu, int n) {
    ExactPlan p;
    const int L = h->cfg.n_layers;
    p.maps = (size_t)n * Tk * Tu * L;
    const int Hs = (Tk + 6 - 7) / 2 + 1, Ws = (Tu + 6 - 7) / 2 + 1;
    p.stem = (size_t)n * Hs * Ws * 64;
    int H = (Hs - 1) / 2 + 1, W = (Ws - 1) / 2 + 1;
    p.big = (size_t)n * H * W * 64;
    for (const auto& b : h->blocks32) {
        int Ho = H, Wo = W;
        if (b.has_sc) {
            const int hs = (H - 1) / b.sc.stride + 1, ws = (W - 1) / b.sc.stride + 1;
            p.big = std::max(p.big, (size_t)n * hs * ws * b.sc.cout);
        }
        for (int j = 0; j < b.nconv; ++j) {
            const auto& c = b.conv[j];
            Ho = (Ho + 2 * (c.k / 2) - c.k) / c.stride + 1;
            Wo = (Wo + 2 * (c.k / 2) - c.k) / c.stride + 1;
            const size_t e = (size_t)n * Ho * Wo * c.cout;
            if (j + 1 < b.nconv) p.small = std::max(p.small, e); else p.big = std::max(p.big, e);
        }
        H = Ho;
        W = Wo;
    }
    return p;
}
}  // namespace

int64_t cbw_kws_project_f32_workspace_bytes(cbw_kws* h, int B, int T) {
    if (!h) return -1;
    const int L = h->cfg.n_layers, D = h->cfg.embedding_dim, U = h->cfg.proj_units;
    const size_t rows = (size_t)L * B * T;
    return (int64_t)(align_up(rows * D * 4) + align_up(rows * (D / 2) * 4) + align_up(rows * U * 4));
}

int cbw_kws_project_f32(cbw_kws* h, const float* x, const float* mask, int B, int T, float* out, float* mask_out,
                        void* ws, int64_t ws_bytes, cbw_stream_t stream) {
    if (!h || !x || !mask || !out || !mask_out) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized || h->stem32.cout == 0) return fail(CBW_ERR_STATE, "cbw_kws_finalize not called (or no fp32 path)");
    if (B <= 0 || T <= 0) return fail(CBW_ERR_INVALID, "B and T must be positive");
    hipStream_t st = (hipStream_t)stream;
    const int L = h->cfg.n_layers, D = h->cfg.embedding_dim, U = h->cfg.proj_units;
    const float eps = 1e-6f;
    if (h->cfg.variant == 0) {
        HIPCHK(cbw_normalize_rows(x, 1, out, 1, 1, B * L, T, D, eps, 0, st));
        HIPCHK(hipMemcpyAsync(mask_out, mask, sizeof(float) * B * L * T, hipMemcpyDeviceToDevice, st));
        return CBW_OK;
    }
    if (ws_bytes < cbw_kws_project_f32_workspace_bytes(h, B, T)) return fail(CBW_ERR_OOM, "workspace too small");
    const size_t rows_l = (size_t)B * T;
    char* p = (char*)ws;
    float* xp = (float*)p; p += align_up(rows_l * L * D * 4);
    float* h1 = (float*)p; p += align_up(rows_l * L * (D / 2) * 4);
    float* h2 = (float*)p;
    HIPCHK(cbw_permute_lbtd_f32(x, xp, B, L, T, D, st));
    for (int l = 0; l < L; ++l) {
        CHK(launch_conv32(h->p1_32[l], xp + (size_t)l * rows_l * D, 1, 1, (int)rows_l, h1 + (size_t)l * rows_l * (D / 2),
                          nullptr, true, st));
        CHK(launch_conv32(h->p2_32[l], h1 + (size_t)l * rows_l * (D / 2), 1, 1, (int)rows_l, h2 + (size_t)l * rows_l * U,
                          nullptr, false, st));
    }
    if (h->cfg.variant == 1) {
        HIPCHK(cbw_normalize_rows(h2, 1, out, 1, L, B, T, U, eps, 1, st));
        HIPCHK(hipMemcpyAsync(mask_out, mask, sizeof(float) * B * L * T, hipMemcpyDeviceToDevice, st));
    } else {
        HIPCHK(cbw_lef_time_project(h2, h->tp_w.as<float>(), h->tp_b.as<float>(), out, 1, mask, mask_out, L, B, T, U,
                                    eps, st));
    }
    return CBW_OK;
}

int64_t cbw_kws_rescore_workspace_bytes(cbw_kws* h, int Tk, int Tu) {
    if (!h || !h->finalized || h->stem32.cout == 0) return -1;
    const ExactPlan p = exact_plan(h, Tk, Tu, EXACT_CHUNK);
    return (int64_t)(align_up(p.maps * 4) + align_up(p.stem * 4) + 3 * align_up(p.big * 4) + 2 * align_up(p.small * 4));
}

}  // extern "C"
namespace {
// channel sums of the fp32 network's conv inputs (cbw_kws_calibrate_bias): point 0 the maps, then per block
// 1 + 3 i its input, 2 + 3 i the first conv's output, 3 + 3 i the second's (bottleneck)
struct ConvInputStats {
    std::vector<int> ch;          // channels per point (0: unused)
    std::vector<size_t> off;      // float offset of point i's [G][C] partial sums in part
    std::vector<double> rows;     // rows summed per point
    float* part = nullptr;        // null: no channel sums
    int G = 0;
    // absolute maxima (the fp8 tier's activation scales): per block i, point 4 i + {0 input, 1 first conv's
    // output, 2 second conv's output, 3 shortcut output}; amax[p * groups + g] = workgroup g's partial
    float* amax = nullptr;
    int add(size_t i, const float* x, int64_t M, hipStream_t st) {
        if (!part) return CBW_OK;
        rows[i] += (double)M;
        HIPCHK(cbw_channel_sum_f32(x, M, ch[i], part + off[i], st));
        return CBW_OK;
    }
    int absmax(size_t p, const float* x, int64_t n, hipStream_t st) {
        if (!amax) return CBW_OK;
        HIPCHK(cbw_absmax_f32(x, n, amax + p * cbw_absmax_groups(), st));
        return CBW_OK;
    }
};

// the fp32 re-scoring network over selected pairs; logits null: no classifier (statistics only)
int rescore_impl(cbw_kws* h, const float* utt, const float* utt_mask, const float* kwd, const float* kwd_mask, int K,
                 int Tk, int Tu, const int32_t* sel, int n_sel, float* logits, void* ws, int64_t ws_bytes,
                 hipStream_t st, ConvInputStats* stats) {
    if (!h->finalized || h->stem32.cout == 0) return fail(CBW_ERR_STATE, "cbw_kws_finalize not called (or no fp32 path)");
    if (K < 0 || n_sel < 0 || n_sel > K || Tk <= 0 || Tu <= 0) return fail(CBW_ERR_INVALID, "bad sizes");
    if (n_sel == 0) return CBW_OK;
    if (ws_bytes < cbw_kws_rescore_workspace_bytes(h, Tk, Tu)) return fail(CBW_ERR_OOM, "workspace too small");
    const int L = h->cfg.n_layers;
    const int E = h->cfg.variant == 0 ? h->cfg.embedding_dim : h->cfg.proj_units;
    const ExactPlan plan = exact_plan(h, Tk, Tu, EXACT_CHUNK);
    char* p = (char*)ws;
    float* maps = (float*)p; p += align_up(plan.maps * 4);
    float* stem = (float*)p; p += align_up(plan.stem * 4);
    float* X = (float*)p; p += align_up(plan.big * 4);
    float* Y = (float*)p; p += align_up(plan.big * 4);
    float* SC = (float*)p; p += align_up(plan.big * 4);
    float* T1 = (float*)p; p += align_up(plan.small * 4);
    float* T2 = (float*)p;
    // a call over all 10 000 pairs enqueues ~19 000 dispatches (313 passes x ~60 launches); under rocprofv3
    // --pmc such a call faulted inside hipLaunchKernel (profiles/r05b_pmc_f32_one_call_sigsegv.log.txt) while the same
    // passes in host-synchronised calls of 512 pairs (~1 000 dispatches each) ran clean.  So one call keeps at most
    // 2 x RESCORE_THROTTLE passes in flight: every RESCORE_THROTTLE passes it records an event and waits on the host
    // for the previous one.  Not while the stream is being captured (the call stays graph-capturable); results
    // unchanged.  Round 6: with 128 passes (~7 700 dispatches) in flight the one-call audit under --pmc still failed
    // (unspecified launch failure, 3 956 dispatches incomplete: profiles/r06b_pmc_f32_one_call_throttle128.log.txt),
    // so the bound is the r05b passes' ~1 000 dispatches.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(st, &cap));
    const bool throttle = cap == hipStreamCaptureStatusNone && n_sel > RESCORE_THROTTLE * EXACT_CHUNK;
    if (throttle)
        for (auto& e : h->throttle_ev)
            if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int pass = 0;
    for (int c0 = 0; c0 < n_sel; c0 += EXACT_CHUNK, ++pass) {
        const int cn = std::min(EXACT_CHUNK, n_sel - c0);
        if (throttle && pass > 0 && pass % RESCORE_THROTTLE == 0) {
            const int k = (pass / RESCORE_THROTTLE) & 1;
            if (pass >= 2 * RESCORE_THROTTLE) HIPCHK(hipEventSynchronize(h->throttle_ev[k]));
            HIPCHK(hipEventRecord(h->throttle_ev[k], st));
        }
        HIPCHK(cbw_sim_f32(kwd, kwd_mask, utt, utt_mask, sel, c0, cn, maps, L, Tk, Tu, E, st));
        if (stats) CHK(stats->add(0, maps, (int64_t)cn * Tk * Tu, st));
        int Hs, Ws;
        CHK(launch_conv32(h->stem32, maps, cn, Tk, Tu, stem, nullptr, true, st, &Hs, &Ws));
        int H = (Hs - 1) / 2 + 1, W = (Ws - 1) / 2 + 1, C = 64;
        HIPCHK(cbw_maxpool_f32(stem, X, cn, Hs, Ws, 64, H, W, st));
        float *x = X, *y = Y;
        size_t bi = 0;
        for (const auto& b : h->blocks32) {
            const float* res = x;
            if (stats) CHK(stats->add(1 + 3 * bi, x, (int64_t)cn * H * W, st));
            if (stats) CHK(stats->absmax(4 * bi, x, (int64_t)cn * H * W * C, st));
            if (b.has_sc) {
                CHK(launch_conv32(b.sc, x, cn, H, W, SC, nullptr, false, st));
                res = SC;
                if (stats) {
                    const int hs = (H - 1) / b.sc.stride + 1, ws2 = (W - 1) / b.sc.stride + 1;
                    CHK(stats->absmax(4 * bi + 3, SC, (int64_t)cn * hs * ws2 * b.sc.cout, st));
                }
            }
            int Ho = H, Wo = W;
            if (b.nconv == 3) {
                int h1, w1;
                CHK(launch_conv32(b.conv[0], x, cn, H, W, T1, nullptr, true, st, &h1, &w1));
                if (stats) CHK(stats->add(2 + 3 * bi, T1, (int64_t)cn * h1 * w1, st));
                if (stats) CHK(stats->absmax(4 * bi + 1, T1, (int64_t)cn * h1 * w1 * b.conv[0].cout, st));
                CHK(launch_conv32(b.conv[1], T1, cn, h1, w1, T2, nullptr, true, st, &Ho, &Wo));
                if (stats) CHK(stats->add(3 + 3 * bi, T2, (int64_t)cn * Ho * Wo, st));
                if (stats) CHK(stats->absmax(4 * bi + 2, T2, (int64_t)cn * Ho * Wo * b.conv[1].cout, st));
                CHK(launch_conv32(b.conv[2], T2, cn, Ho, Wo, y, res, true, st));
            } else {
                CHK(launch_conv32(b.conv[0], x, cn, H, W, T1, nullptr, true, st, &Ho, &Wo));
                if (stats) CHK(stats->add(2 + 3 * bi, T1, (int64_t)cn * Ho * Wo, st));
                CHK(launch_conv32(b.conv[1], T1, cn, Ho, Wo, y, res, true, st));
            }
            std::swap(x, y);
            H = Ho;
            W = Wo;
            C = b.conv[b.nconv - 1].cout;
            ++bi;
        }
        if (logits)
            HIPCHK(cbw_pool_fc_f32(x, h->fc_w.as<float>(), h->fc_b.as<float>(), sel, c0, cn, logits, H * W, C, st));
    }
    return CBW_OK;
}

float bf16_round_host(float v) {
    const uint32_t u = (uint32_t)f2bf_host(v) << 16;
    float r;
    std::memcpy(&r, &u, 4);
    return r;
}

// the folded fp32 bias of a conv plus, with input channel means m, the bias correction
// sum_{kh, kw, c} m[c] (w - bf16(w)): the mean shift the bf16 weights put on each output channel
int corrected_bias(const ParamStore& ps, const std::string& prefix, int cin, int cout, int k, const double* m,
                   std::vector<double>& b) {
    std::vector<float> w, sh;
    CHK(fold_conv_host(ps, prefix, cin, cout, k, w, sh));
    b.assign(sh.begin(), sh.end());
    if (!m) return CBW_OK;
    const size_t taps = (size_t)k * k;
    for (int o = 0; o < cout; ++o) {
        double s = 0.0;
        for (size_t t = 0; t < taps; ++t) {
            const float* row = &w[((size_t)o * taps + t) * cin];
            for (int c = 0; c < cin; ++c) s += m[c] * ((double)row[c] - (double)bf16_round_host(row[c]));
        }
        b[o] += s;
    }
    return CBW_OK;
}

// rewrite a bias vector in place (same allocation: captured graphs and in-flight plans keep their pointers)
int overwrite_bias(DevBuf& d, const std::vector<double>& v) {
    if (d.bytes != v.size() * sizeof(float)) return fail(CBW_ERR_STATE, "bias size mismatch");
    const std::vector<float> f(v.begin(), v.end());
    HIPCHK(hipMemcpy(d.p, f.data(), d.bytes, hipMemcpyHostToDevice));
    return CBW_OK;
}

// the bf16 scoring network's biases from the parameters, corrected with the conv-input means m (ConvInputStats
// points) or, m null, as folded (cbw_kws_finalize's values)
int apply_bias_correction(cbw_kws* h, const std::vector<std::vector<double>>* m) {
    // the folded biases are read by scoring launches on any stream: drain the device before rewriting them
    HIPCHK(hipDeviceSynchronize());
    auto mean = [&](size_t i) -> const double* { return m && !(*m)[i].empty() ? (*m)[i].data() : nullptr; };
    std::vector<double> b, b2;
    CHK(corrected_bias(h->ps, "model.feature_extractor.embedder.embedder", h->cfg.n_layers, 64, 7, mean(0), b));
    CHK(overwrite_bias(h->stem_b, b));
    for (size_t bi = 0; bi < h->blocks.size(); ++bi) {
        BlockW& blk = h->blocks[bi];
        const double* in[3] = {mean(1 + 3 * bi), mean(2 + 3 * bi), mean(3 + 3 * bi)};
        if (blk.has_sc && !blk.fused_sc) {
            CHK(corrected_bias(h->ps, blk.prefix + ".shortcut", blk.sc.cin, blk.sc.cout, 1, in[0], b));
            CHK(overwrite_bias(blk.sc.b, b));
        }
        for (int j = 0; j < blk.nconv; ++j) {
            const ConvW& c = blk.conv[j];
            CHK(corrected_bias(h->ps, blk.prefix + ".layer." + std::to_string(j), c.cin, c.cout, c.k, in[j], b));
            if (j == 2 && blk.fused_sc) {   // + the shortcut's bias and correction (K-concatenated conv)
                CHK(corrected_bias(h->ps, blk.prefix + ".shortcut", blk.sc.cin, blk.sc.cout, 1, in[0], b2));
                for (size_t o = 0; o < b.size(); ++o) b[o] += b2[o];
            }
            CHK(overwrite_bias(blk.conv[j].b, b));
        }
    }
    return CBW_OK;
}
}  // namespace
extern "C" {

int cbw_kws_rescore(cbw_kws* h, const float* utt, const float* utt_mask, const float* kwd, const float* kwd_mask, int K,
                    int Tk, int Tu, const int32_t* sel, int n_sel, float* logits, void* ws, int64_t ws_bytes,
                    cbw_stream_t stream) {
    if (!h || !utt || !utt_mask || !kwd || !kwd_mask || !logits || (n_sel > 0 && !sel))
        return fail(CBW_ERR_INVALID, "null argument");
    return rescore_impl(h, utt, utt_mask, kwd, kwd_mask, K, Tk, Tu, sel, n_sel, logits, ws, ws_bytes,
                        (hipStream_t)stream, nullptr);
}

int cbw_kws_set_score_offset(cbw_kws* h, const float* offset) {
    if (!h || !offset) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized || h->fc_b16.bytes != 2 * sizeof(float)) return fail(CBW_ERR_STATE, "cbw_kws_finalize not called");
    int rc;
    const auto* fb = h->ps.get("model.classifier.1.bias", 2, &rc);
    if (!fb) return rc;
    const float b[2] = {(*fb)[0] + offset[0], (*fb)[1] + offset[1]};
    // the bias is read by scoring launches on any stream: drain the device before overwriting it in place
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(h->fc_b16.p, b, sizeof(b), hipMemcpyHostToDevice));
    return CBW_OK;
}

int cbw_kws_calibrate_bias(cbw_kws* h, const float* utt, const float* utt_mask, const float* kwd, const float* kwd_mask,
                           int K, int Tk, int Tu, const int32_t* sel, int n_sel, void* ws, int64_t ws_bytes,
                           cbw_stream_t stream) {
    if (!h) return fail(CBW_ERR_INVALID, "null handle");
    if (!h->finalized || h->stem32.cout == 0) return fail(CBW_ERR_STATE, "cbw_kws_finalize not called (or no fp32 path)");
    hipStream_t st = (hipStream_t)stream;
    if (n_sel == 0) {   // back to the folded biases (and no logit offset)
        HIPCHK(hipDeviceSynchronize());
        const float zero2[2] = {0.f, 0.f};
        CHK(cbw_kws_set_score_offset(h, zero2));
        return apply_bias_correction(h, nullptr);
    }
    if (!utt || !utt_mask || !kwd || !kwd_mask || !sel) return fail(CBW_ERR_INVALID, "null argument");
    if (h->blocks.size() != h->blocks32.size()) return fail(CBW_ERR_STATE, "fp32 and bf16 networks differ");
    ConvInputStats s;
    s.G = cbw_channel_sum_groups();
    s.ch.push_back(h->cfg.n_layers);
    for (const auto& b : h->blocks32) {
        s.ch.push_back(b.conv[0].cin);
        s.ch.push_back(b.conv[0].cout);
        s.ch.push_back(b.nconv == 3 ? b.conv[1].cout : 0);
    }
    size_t tot = 0;
    for (int c : s.ch) { s.off.push_back(tot); tot += (size_t)s.G * c; }
    s.rows.assign(s.ch.size(), 0.0);
    DevBuf part;
    CHK(part.alloc(tot * sizeof(float)));
    s.part = part.as<float>();
    HIPCHK(hipMemsetAsync(part.p, 0, tot * sizeof(float), st));
    CHK(rescore_impl(h, utt, utt_mask, kwd, kwd_mask, K, Tk, Tu, sel, n_sel, nullptr, ws, ws_bytes, st, &s));
    HIPCHK(hipStreamSynchronize(st));
    std::vector<float> host(tot);
    HIPCHK(hipMemcpy(host.data(), part.p, tot * sizeof(float), hipMemcpyDeviceToHost));
    std::vector<std::vector<double>> m(s.ch.size());
    for (size_t i = 0; i < s.ch.size(); ++i) {
        if (!s.ch[i] || s.rows[i] <= 0) continue;
        m[i].assign(s.ch[i], 0.0);
        for (int g = 0; g < s.G; ++g)
            for (int c = 0; c < s.ch[i]; ++c) m[i][c] += host[s.off[i] + (size_t)g * s.ch[i] + c];
        for (double& v : m[i]) v /= s.rows[i];
    }
    return apply_bias_correction(h, &m);
}

int cbw_kws_calibrate_fp8(cbw_kws* h, const float* utt, const float* utt_mask, const float* kwd, const float* kwd_mask,
                          int K, int Tk, int Tu, const int32_t* sel, int n_sel, float margin, void* ws, int64_t ws_bytes,
                          cbw_stream_t stream) {
    if (!h || !utt || !utt_mask || !kwd || !kwd_mask || !sel || n_sel <= 0) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized || h->stem32.cout == 0) return fail(CBW_ERR_STATE, "cbw_kws_finalize not called (or no fp32 path)");
    if (h->cfg.resnet_depth != 50 || h->blocks.size() != h->blocks32.size())
        return fail(CBW_ERR_INVALID, "the fp8 tier covers ResNet-50 (bottleneck stages 2-4)");
    if (!(margin > 0.f)) return fail(CBW_ERR_INVALID, "margin must be positive");
    hipStream_t st = (hipStream_t)stream;
    const size_t nb = h->blocks32.size();
    const char* bc = getenv("CBW_FP8_BIAS_CORR");   // 0: the folded biases (A/B)
    const bool bias_corr = !(bc && atoi(bc) == 0);
    const int G = cbw_absmax_groups();
    DevBuf amax;
    CHK(amax.alloc(nb * 4 * G * sizeof(float)));
    HIPCHK(hipMemsetAsync(amax.p, 0, nb * 4 * G * sizeof(float), st));
    ConvInputStats s;
    s.amax = amax.as<float>();
    // + the conv inputs' channel sums (the bias correction of the e4m3 weights), points as cbw_kws_calibrate_bias
    s.G = cbw_channel_sum_groups();
    s.ch.push_back(h->cfg.n_layers);
    for (const auto& b : h->blocks32) {
        s.ch.push_back(b.conv[0].cin);
        s.ch.push_back(b.conv[0].cout);
        s.ch.push_back(b.nconv == 3 ? b.conv[1].cout : 0);
    }
    size_t tot = 0;
    for (int c : s.ch) { s.off.push_back(tot); tot += (size_t)s.G * c; }
    s.rows.assign(s.ch.size(), 0.0);
    DevBuf part;
    CHK(part.alloc(tot * sizeof(float)));
    s.part = part.as<float>();
    HIPCHK(hipMemsetAsync(part.p, 0, tot * sizeof(float), st));
    CHK(rescore_impl(h, utt, utt_mask, kwd, kwd_mask, K, Tk, Tu, sel, n_sel, nullptr, ws, ws_bytes, st, &s));
    HIPCHK(hipStreamSynchronize(st));
    std::vector<float> host(nb * 4 * G);
    HIPCHK(hipMemcpy(host.data(), amax.p, host.size() * sizeof(float), hipMemcpyDeviceToHost));
    std::vector<float> sums(tot);
    HIPCHK(hipMemcpy(sums.data(), part.p, tot * sizeof(float), hipMemcpyDeviceToHost));
    std::vector<std::vector<double>> mean(s.ch.size());
    for (size_t i = 0; i < s.ch.size(); ++i) {
        if (!s.ch[i] || s.rows[i] <= 0) continue;
        mean[i].assign(s.ch[i], 0.0);
        for (int g = 0; g < s.G; ++g)
            for (int c = 0; c < s.ch[i]; ++c) mean[i][c] += sums[s.off[i] + (size_t)g * s.ch[i] + c];
        for (double& v : mean[i]) v /= s.rows[i];
    }
    auto mp = [&](size_t i) -> const double* { return bias_corr && !mean[i].empty() ? mean[i].data() : nullptr; };
    auto scale = [&](size_t p) {
        float m = 0.f;
        for (int g = 0; g < G; ++g) m = std::max(m, host[p * G + g]);
        return m > 0.f ? m * margin / 448.f : 1.f;
    };
    int first = -1;
    for (size_t i = 0; i < nb; ++i)
        if (h->blocks[i].stage >= 2) { first = (int)i; break; }
    if (first < 0) return fail(CBW_ERR_STATE, "no stage-2 blocks");
    std::vector<BlockF8> b8(nb - first);
    for (size_t i = first; i < nb; ++i) {
        const BlockW32& b = h->blocks32[i];
        BlockF8& q = b8[i - first];
        if (b.nconv != 3) return fail(CBW_ERR_INVALID, "bottleneck blocks only");
        const std::string& p = h->blocks[i].prefix;
        q.s_x = scale(4 * i); q.s_t1 = scale(4 * i + 1); q.s_t2 = scale(4 * i + 2);
        q.has_sc = b.has_sc;
        if (b.has_sc) {
            q.s_sc = scale(4 * i + 3);
            CHK(load_conv_f8(h->ps, p + ".shortcut", b.sc.cin, b.sc.cout, 1, b.sc.stride, false, q.s_x, q.sc,
                             mp(1 + 3 * i)));
        }
        CHK(load_conv_f8(h->ps, p + ".layer.0", b.conv[0].cin, b.conv[0].cout, 1, 1, true, q.s_x, q.conv[0],
                         mp(1 + 3 * i)));
        CHK(load_conv_f8(h->ps, p + ".layer.1", b.conv[1].cin, b.conv[1].cout, 3, b.conv[1].stride, true, q.s_t1,
                         q.conv[1], mp(2 + 3 * i)));
        CHK(load_conv_f8(h->ps, p + ".layer.2", b.conv[2].cin, b.conv[2].cout, 1, 1, true, q.s_t2, q.conv[2],
                         mp(3 + 3 * i)));
        q.out_bf16 = i + 1 == nb;
        q.s_out = q.out_bf16 ? 1.f : scale(4 * (i + 1));
    }
    HIPCHK(hipDeviceSynchronize());   // setup-time: no scoring may be in flight on any stream while the tier changes
    h->blocks8 = std::move(b8);
    h->f8_first = first;
    h->f8_in_scale = h->blocks8[0].s_x;
    return CBW_OK;
}

int x3_stem32() {   // CBW_X3_STEM32=1: the compensated tier's stem in fp32 (conv_f32 + max-pool + split)
    const char* e = getenv("CBW_X3_STEM32");
    return e ? atoi(e) : 0;
}

// pairs per compensated-tier pass (CBW_X3_CHUNK overrides; read once per process).  bench.py, 855 band pairs
// per clip: 128 -> 58.4 ms, 256 -> 55.8, 512 -> 51.9, 1024 -> 51.2 (workspace ~21 MB per pair at LEF maps)
int x3_chunk() {
    static const int c = [] {
        const char* e = getenv("CBW_X3_CHUNK");
        const int v = e ? atoi(e) : 512;
        return v > 0 ? v : 512;
    }();
    return c;
}

int64_t cbw_kws_rescore_x3_workspace_bytes(cbw_kws* h, int Tk, int Tu) {
    if (!h || !h->finalized || h->stem32.cout == 0 || h->blocks3.empty() || Tk <= 0 || Tu <= 0) return -1;
    const ExactPlan p = exact_plan(h, Tk, Tu, x3_chunk());
    return (int64_t)(align_up(p.maps * 4) + align_up(p.stem * 4) + 2 * align_up(p.big * 4) + 2 * align_up(p.big * 4) +
                     2 * align_up(p.small * 4));
}

int cbw_kws_rescore_x3(cbw_kws* h, const float* utt, const float* utt_mask, const float* kwd, const float* kwd_mask,
                       int K, int Tk, int Tu, const int32_t* sel, int n_sel, float* logits, void* ws, int64_t ws_bytes,
                       cbw_stream_t stream) {
    if (!h || !utt || !utt_mask || !kwd || !kwd_mask || !logits || (n_sel > 0 && !sel))
        return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized || h->stem32.cout == 0 || h->blocks3.empty())
        return fail(CBW_ERR_STATE, "cbw_kws_finalize not called (or no re-scoring path)");
    if (K < 0 || n_sel < 0 || n_sel > K || Tk <= 0 || Tu <= 0) return fail(CBW_ERR_INVALID, "bad sizes");
    if (n_sel == 0) return CBW_OK;
    if (ws_bytes < cbw_kws_rescore_x3_workspace_bytes(h, Tk, Tu)) return fail(CBW_ERR_OOM, "workspace too small");
    hipStream_t st = (hipStream_t)stream;
    const int L = h->cfg.n_layers;
    const int E = h->cfg.variant == 0 ? h->cfg.embedding_dim : h->cfg.proj_units;
    const ExactPlan plan = exact_plan(h, Tk, Tu, x3_chunk());
    char* p = (char*)ws;
    float* maps = (float*)p; p += align_up(plan.maps * 4);
    float* stem = (float*)p; p += align_up(plan.stem * 4);
    float* X32 = (float*)p; p += align_up(plan.big * 4);     // stem/max-pool output, then the network output
    float* SC32 = (float*)p; p += align_up(plan.big * 4);    // projection shortcuts
    uint16_t* X3 = (uint16_t*)p; p += align_up(plan.big * 4);   // [hi | lo] activations, 4 bytes per element
    uint16_t* Y3 = (uint16_t*)p; p += align_up(plan.big * 4);
    uint16_t* T1 = (uint16_t*)p; p += align_up(plan.small * 4);
    uint16_t* T2 = (uint16_t*)p;
    const void* zp = h->zero.p;
    const size_t nb = h->blocks3.size();
    const int X3_CHUNK = x3_chunk();
    for (int c0 = 0; c0 < n_sel; c0 += X3_CHUNK) {
        const int cn = std::min(X3_CHUNK, n_sel - c0);
        // similarity maps in fp32, then the stem + max-pool: compensated bf16 in one pass (maps split into
        // [hi | hi | lo] channels of an NHWC16 image, cbw_stem16_pool_x3; CBW_X3_STEM32=1 or 3 L > 16: the fp32
        // stem, max-pool and split)
        HIPCHK(cbw_sim_f32(kwd, kwd_mask, utt, utt_mask, sel, c0, cn, maps, L, Tk, Tu, E, st));
        const int Hs = (Tk + 2 * 3 - 7) / 2 + 1, Ws = (Tu + 2 * 3 - 7) / 2 + 1;
        int H = (Hs - 1) / 2 + 1, W = (Ws - 1) / 2 + 1, C = 64;
        if (h->stem16x3_w.p && !x3_stem32()) {
            uint16_t* m16 = (uint16_t*)stem;   // [cn][Tk][Tu][16] bf16 fits the fp32 stem buffer
            HIPCHK(cbw_maps_split16(maps, m16, cn, L, Tk, Tu, st));
            HIPCHK(cbw_stem16_pool_x3(m16, h->stem16x3_w.as<uint16_t>(), h->stem32.b.as<float>(), X3, cn, Tk, Tu, Hs,
                                      Ws, H, W, st));
        } else {
            int hs2, ws2;
            CHK(launch_conv32(h->stem32, maps, cn, Tk, Tu, stem, nullptr, true, st, &hs2, &ws2));
            HIPCHK(cbw_maxpool_f32(stem, X32, cn, Hs, Ws, 64, H, W, st));
            HIPCHK(cbw_split3(X32, X3, (int64_t)cn * H * W, 64, st));
        }
        uint16_t *x3 = X3, *y3 = Y3;
        for (size_t bi = 0; bi < nb; ++bi) {
            const auto& b = h->blocks3[bi];
            const void* res = x3;   // identity shortcut: the block input's [hi | lo]
            bool res_split = true;
            if (b.has_sc) {
                CHK(launch_conv_x3(b.sc, x3, cn, H, W, SC32, nullptr, nullptr, false, CBW_EPI_OUT_F32, zp, st, nullptr,
                                   nullptr, &h->prof));
                res = SC32;
                res_split = false;
            }
            float* out32 = bi + 1 == nb ? X32 : nullptr;   // fp32 network output for the pool + classifier
            int Ho = H, Wo = W;
            if (b.nconv == 3) {
                int h1, w1;
                CHK(launch_conv_x3(b.conv[0], x3, cn, H, W, T1, nullptr, nullptr, false, CBW_EPI_SPLIT3, zp, st, &h1,
                                   &w1, &h->prof));
                CHK(launch_conv_x3(b.conv[1], T1, cn, h1, w1, T2, nullptr, nullptr, false, CBW_EPI_SPLIT3, zp, st, &Ho,
                                   &Wo, &h->prof));
                CHK(launch_conv_x3(b.conv[2], T2, cn, Ho, Wo, y3, out32, res, res_split, CBW_EPI_SPLIT3, zp, st, nullptr,
                                   nullptr, &h->prof));
            } else {
                CHK(launch_conv_x3(b.conv[0], x3, cn, H, W, T1, nullptr, nullptr, false, CBW_EPI_SPLIT3, zp, st, &Ho,
                                   &Wo, &h->prof));
                CHK(launch_conv_x3(b.conv[1], T1, cn, Ho, Wo, y3, out32, res, res_split, CBW_EPI_SPLIT3, zp, st, nullptr,
                                   nullptr, &h->prof));
            }
            std::swap(x3, y3);
            H = Ho;
            W = Wo;
            C = b.conv[b.nconv - 1].cout;
        }
        HIPCHK(cbw_pool_fc_f32(X32, h->fc_w.as<float>(), h->fc_b.as<float>(), sel, c0, cn, logits, H * W, C, st));
    }
    return CBW_OK;
}

int cbw_kws_spot(const float* logits, const float* ghost, int K, float thr, int mode, float* prob, int32_t* idx,
                 int32_t* n, cbw_stream_t stream) {
    if (!idx || !n || K < 0 || (K > 0 && !logits)) return fail(CBW_ERR_INVALID, "bad arguments");
    if (K == 0) {
        HIPCHK(hipMemsetAsync(n, 0, sizeof(int32_t), (hipStream_t)stream));
        return CBW_OK;
    }
    if (mode != 0 && mode != 1) return fail(CBW_ERR_INVALID, "cbw_kws_spot: mode must be 0 (threshold) or 1 (argmax)");
    HIPCHK(cbw_spot(logits, ghost, K, thr, 0.f, mode, prob, idx, n, (hipStream_t)stream));
    return CBW_OK;
}

int64_t cbw_checksum_workspace_bytes(void) { return cbw_checksum_scratch_bytes(); }

int cbw_checksum(const void* data, int64_t bytes, uint64_t* out, void* ws, int64_t ws_bytes, cbw_stream_t stream) {
    if (!out || !ws || bytes < 0 || (bytes > 0 && !data)) return fail(CBW_ERR_INVALID, "null argument");
    if ((uintptr_t)data & 15) return fail(CBW_ERR_INVALID, "cbw_checksum: data must be 16-byte aligned");
    if (ws_bytes < cbw_checksum_scratch_bytes()) return fail(CBW_ERR_OOM, "checksum workspace too small");
    HIPCHK(cbw_checksum64(data, bytes, out, (uint64_t*)ws, (hipStream_t)stream));
    return CBW_OK;
}

int cbw_kws_band(const float* logits, const float* ghost, int K, float thr, float band, int32_t* idx, int32_t* n,
                 cbw_stream_t stream) {
    if (!idx || !n || K < 0 || (K > 0 && !logits) || !(band >= 0.f)) return fail(CBW_ERR_INVALID, "bad arguments");
    if (K == 0) {
        HIPCHK(hipMemsetAsync(n, 0, sizeof(int32_t), (hipStream_t)stream));
        return CBW_OK;
    }
    HIPCHK(cbw_spot(logits, ghost, K, thr, band, 2, nullptr, idx, n, (hipStream_t)stream));
    return CBW_OK;
}
int cbw_kws_band_scaled(const float* logits, const float* ghost, int K, float thr, float coef, int32_t* idx, int32_t* n,
                        cbw_stream_t stream) {
    if (!idx || !n || K < 0 || (K > 0 && !logits) || !(coef >= 0.f)) return fail(CBW_ERR_INVALID, "bad arguments");
    if (K == 0) {
        HIPCHK(hipMemsetAsync(n, 0, sizeof(int32_t), (hipStream_t)stream));
        return CBW_OK;
    }
    HIPCHK(cbw_spot(logits, ghost, K, thr, coef, 3, nullptr, idx, n, (hipStream_t)stream));
    return CBW_OK;
}

// ------------------------------------------------------------------ mel
namespace {
int mel_impl(const float* pcm, int64_t n, int n_mel, float* out, uint16_t* packed, int cpad, void* ws,
             cbw_stream_t stream, bool long_form) {
    static thread_local std::map<std::pair<int, int>, std::shared_ptr<DevBuf>> tables;   // (device, n_mel) -> [filters|twiddle]
    if (!pcm || !out || !ws || n < 0 || n_mel <= 0 || n_mel > 256) return fail(CBW_ERR_INVALID, "bad arguments");
    if (packed && (cpad < n_mel || cpad % 64)) return fail(CBW_ERR_INVALID, "cpad must be >= n_mel and a multiple of 64");
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    auto key = std::make_pair(dev, n_mel);
    auto it = tables.find(key);
    if (it == tables.end()) {
        // slaney mel filter bank (HF audio_utils.mel_filter_bank(norm='slaney', mel_scale='slaney')), [201][n_mel]
        const int nf = 201;
        auto hz2mel = [](double f) { return f >= 1000.0 ? 15.0 + std::log(f / 1000.0) * (27.0 / std::log(6.4)) : 3.0 * f / 200.0; };
        auto mel2hz = [](double m) { return m >= 15.0 ? 1000.0 * std::exp(std::log(6.4) / 27.0 * (m - 15.0)) : 200.0 * m / 3.0; };
        std::vector<double> ff(n_mel + 2);
        const double m0 = hz2mel(0.0), m1 = hz2mel(8000.0);
        for (int i = 0; i < n_mel + 2; ++i) ff[i] = mel2hz(m0 + (m1 - m0) * i / (n_mel + 1));
        std::vector<float> tab((size_t)nf * n_mel + 800);
        for (int f = 0; f < nf; ++f) {
            const double fr = 8000.0 * f / (nf - 1);
            for (int m = 0; m < n_mel; ++m) {
                const double down = (fr - ff[m]) / (ff[m + 1] - ff[m]);
                const double up = (ff[m + 2] - fr) / (ff[m + 2] - ff[m + 1]);
                const double v = std::max(0.0, std::min(down, up)) * 2.0 / (ff[m + 2] - ff[m]);
                tab[(size_t)f * n_mel + m] = (float)v;
            }
        }
        for (int k = 0; k < 400; ++k) {
            tab[(size_t)nf * n_mel + k] = (float)std::cos(2.0 * M_PI * k / 400.0);
            tab[(size_t)nf * n_mel + 400 + k] = (float)-std::sin(2.0 * M_PI * k / 400.0);
        }
        auto buf = std::make_shared<DevBuf>();
        CHK(buf->upload(tab));
        it = tables.emplace(key, buf).first;
    }
    const float* filters = it->second->as<float>();
    const float* tw = filters + (size_t)201 * n_mel;
    hipStream_t st = (hipStream_t)stream;
    if (long_form) {
        const int frames = (int)(n / 160);
        HIPCHK(cbw_mel_frames(pcm, (int)n, filters, tw, out, n_mel, st, (int)n, frames));
        HIPCHK(cbw_mel_finish(out, n_mel, (float*)ws, nullptr, 0, st, frames));
        return CBW_OK;
    }
    HIPCHK(cbw_mel_frames(pcm, (int)std::min<int64_t>(n, 480000), filters, tw, out, n_mel, st));
    HIPCHK(cbw_mel_finish(out, n_mel, (float*)ws, packed, packed ? cpad : 0, st));
    return CBW_OK;
}
}  // namespace

int cbw_mel(const float* pcm, int64_t n, int n_mel, float* out, uint16_t* packed, int cpad, void* ws,
            cbw_stream_t stream) {
    return mel_impl(pcm, n, n_mel, out, packed, cpad, ws, stream, false);
}

int cbw_mel_long(const float* pcm, int64_t n, int n_mel, float* out, void* ws, cbw_stream_t stream) {
    if (n < 400 || n > 0x7fffffffLL) return fail(CBW_ERR_INVALID, "cbw_mel_long: 400 <= n_samples < 2^31");
    return mel_impl(pcm, n, n_mel, out, nullptr, 0, ws, stream, true);
}



// ------------------------------------------------------------------ encoder
int cbw_encoder_create(const cbw_encoder_config* cfg, cbw_encoder** out) {
    if (!cfg || !out) return fail(CBW_ERR_INVALID, "null argument");
    if (cfg->n_heads < 1 || cfg->d_model % 128 || cfg->d_model / cfg->n_heads != 64 || cfg->ffn_dim % 128 ||
        cfg->n_layers < 1)
        return fail(CBW_ERR_INVALID, "encoder needs d_model % 128 == 0, head_dim 64, ffn_dim % 128 == 0");
    auto h = std::make_unique<cbw_encoder>();
    h->cfg = *cfg;
    h->cpad = (cfg->n_mel + 63) / 64 * 64;
    CHK(h->zero.alloc(256));
    HIPCHK(hipMemset(h->zero.p, 0, 256));
    *out = h.release();
    return CBW_OK;
}

int cbw_encoder_destroy(cbw_encoder* h) {
    delete h;
    return CBW_OK;
}

int cbw_encoder_set_param(cbw_encoder* h, const char* name, const float* host, int64_t numel) {
    if (!h) return fail(CBW_ERR_INVALID, "null handle");
    h->finalized = false;
    return h->ps.set(name, host, numel);
}

namespace {
int upload_vec(const ParamStore& ps, const std::string& n, size_t numel, DevBuf& dst) {
    int rc;
    const auto* v = ps.get(n, numel, &rc);
    if (!v) return rc;
    return dst.upload(*v);
}
int upload_linear(const ParamStore& ps, const std::string& n, int cout, int cin, bool has_bias, ConvW& c,
                  float scale = 1.0f) {
    int rc;
    const auto* w = ps.get(n + ".weight", (size_t)cout * cin, &rc);
    if (!w) return rc;
    c.cin = cin; c.cout = cout; c.k = 1; c.stride = 1; c.relu = false;
    std::vector<float> ws(*w);
    for (auto& x : ws) x *= scale;
    CHK(c.w.upload(to_bf16(ws)));
    std::vector<float> b(cout, 0.f);
    if (has_bias) {
        const auto* bv = ps.get(n + ".bias", cout, &rc);
        if (!bv) return rc;
        for (int i = 0; i < cout; ++i) b[i] = (*bv)[i] * scale;
    }
    return c.b.upload(b);
}
}  // namespace

int cbw_encoder_finalize(cbw_encoder* h) {
    if (!h) return fail(CBW_ERR_INVALID, "null handle");
    const int D = h->cfg.d_model, F = h->cfg.ffn_dim, nm = h->cfg.n_mel, cp = h->cpad;
    int rc;
    // conv1 [D][n_mel][3] -> [D][1][3][cpad]; conv2 [D][D][3] -> [D][1][3][D]
    {
        const auto* w = h->ps.get("conv1.weight", (size_t)D * nm * 3, &rc); if (!w) return rc;
        std::vector<float> o((size_t)D * 3 * cp, 0.f);
        for (int co = 0; co < D; ++co)
            for (int ci = 0; ci < nm; ++ci)
                for (int k = 0; k < 3; ++k) o[((size_t)co * 3 + k) * cp + ci] = (*w)[((size_t)co * nm + ci) * 3 + k];
        h->conv1.cin = cp; h->conv1.cout = D; h->conv1.k = 3;
        CHK(h->conv1.w.upload(to_bf16(o)));
        CHK(upload_vec(h->ps, "conv1.bias", D, h->conv1.b));
        const auto* w2 = h->ps.get("conv2.weight", (size_t)D * D * 3, &rc); if (!w2) return rc;
        std::vector<float> o2((size_t)D * 3 * D);
        for (int co = 0; co < D; ++co)
            for (int ci = 0; ci < D; ++ci)
                for (int k = 0; k < 3; ++k) o2[((size_t)co * 3 + k) * D + ci] = (*w2)[((size_t)co * D + ci) * 3 + k];
        h->conv2.cin = D; h->conv2.cout = D; h->conv2.k = 3;
        CHK(h->conv2.w.upload(to_bf16(o2)));
        CHK(upload_vec(h->ps, "conv2.bias", D, h->conv2.b));
    }
    CHK(upload_vec(h->ps, "embed_positions.weight", (size_t)1500 * D, h->pos));
    h->layers.clear();
    h->layers.resize(h->cfg.n_layers);
    const float qscale = 1.0f / std::sqrt(64.0f);
    for (int i = 0; i < h->cfg.n_layers; ++i) {
        auto& L = h->layers[i];
        const std::string p = "layers." + std::to_string(i);
        CHK(upload_vec(h->ps, p + ".self_attn_layer_norm.weight", D, L.ln1_g));
        CHK(upload_vec(h->ps, p + ".self_attn_layer_norm.bias", D, L.ln1_b));
        CHK(upload_vec(h->ps, p + ".final_layer_norm.weight", D, L.ln2_g));
        CHK(upload_vec(h->ps, p + ".final_layer_norm.bias", D, L.ln2_b));
        // fused QKV [3D][D]: q (scaled by hd^-1/2, HF WhisperAttention.scaling) | k (no bias) | v
        {
            const auto* wq = h->ps.get(p + ".self_attn.q_proj.weight", (size_t)D * D, &rc); if (!wq) return rc;
            const auto* wk = h->ps.get(p + ".self_attn.k_proj.weight", (size_t)D * D, &rc); if (!wk) return rc;
            const auto* wv = h->ps.get(p + ".self_attn.v_proj.weight", (size_t)D * D, &rc); if (!wv) return rc;
            const auto* bq = h->ps.get(p + ".self_attn.q_proj.bias", D, &rc); if (!bq) return rc;
            const auto* bv = h->ps.get(p + ".self_attn.v_proj.bias", D, &rc); if (!bv) return rc;
            std::vector<float> w((size_t)3 * D * D), b((size_t)3 * D, 0.f);
            for (size_t j = 0; j < (size_t)D * D; ++j) {
                w[j] = (*wq)[j] * qscale;
                w[(size_t)D * D + j] = (*wk)[j];
                w[(size_t)2 * D * D + j] = (*wv)[j];
            }
            for (int j = 0; j < D; ++j) { b[j] = (*bq)[j] * qscale; b[2 * D + j] = (*bv)[j]; }
            L.qkv.cin = D; L.qkv.cout = 3 * D; L.qkv.k = 1;
            CHK(L.qkv.w.upload(to_bf16(w)));
            CHK(L.qkv.b.upload(b));
        }
        CHK(upload_linear(h->ps, p + ".self_attn.out_proj", D, D, true, L.out));
        CHK(upload_linear(h->ps, p + ".fc1", F, D, true, L.fc1));
        CHK(upload_linear(h->ps, p + ".fc2", D, F, true, L.fc2));
    }
    CHK(upload_vec(h->ps, "layer_norm.weight", D, h->lnf_g));
    CHK(upload_vec(h->ps, "layer_norm.bias", D, h->lnf_b));
    h->finalized = true;
    return CBW_OK;
}

}  // extern "C"
namespace {
bool encoder_splitk_enabled() {   // CBW_ENC_SPLITK=0 runs the out-projection / fc2 GEMMs unsplit (A/B experiments)
    const char* e = getenv("CBW_ENC_SPLITK");
    return !(e && atoi(e) == 0);
}
// K-split of the encoder's few-tile GEMMs (out-projection, fc2: M = B x 1500 rows, N = d_model): the factor
// cbw_conv_splitk_factor picks for each, and the fp32 partial-sum floats it needs
int64_t encoder_splitk_floats(const cbw_encoder* h, int B) {
    if (!encoder_splitk_enabled()) return 0;
    const int D = h->cfg.d_model, F = h->cfg.ffn_dim, M = B * 1500;
    int64_t n = 0;
    for (int K : {D, F}) {
        ConvArgs a{};
        a.KH = a.KW = 1; a.Cin = K; a.Cout = D; a.M = M;
        const int S = cbw_conv_splitk_factor(a);
        if (S > 1) n = std::max<int64_t>(n, (int64_t)S * M * D);
    }
    return n;
}
}  // namespace
extern "C" {

int64_t cbw_encoder_workspace_bytes(cbw_encoder* h, int B) {
    if (!h || B <= 0) return -1;
    const size_t D = h->cfg.d_model, F = h->cfg.ffn_dim, T = 1500;
    return (int64_t)(align_up(B * T * D * 4) + align_up(B * 3000 * D * 2) + align_up(B * T * D * 2) +
                     align_up(B * T * 3 * D * 2) + align_up(B * T * D * 2) + align_up(B * T * F * 2) +
                     align_up((size_t)encoder_splitk_floats(h, B) * 4));
}

int cbw_encoder_hs(cbw_encoder* h, const uint16_t* mel, int B, const int32_t* layer_ids, int n_ids, int normalize,
                   float* hs, void* ws, int64_t ws_bytes, cbw_stream_t stream) {
    if (!h || !mel || !layer_ids || !hs || B <= 0 || n_ids <= 0) return fail(CBW_ERR_INVALID, "bad arguments");
    if (!h->finalized) return fail(CBW_ERR_STATE, "cbw_encoder_finalize not called");
    if (ws_bytes < cbw_encoder_workspace_bytes(h, B)) return fail(CBW_ERR_OOM, "encoder workspace too small");
    const int N = h->cfg.n_layers, D = h->cfg.d_model, T = 1500, M = B * T, H = h->cfg.n_heads;
    int max_id = 0;
    for (int j = 0; j < n_ids; ++j) {
        if (layer_ids[j] < 0 || layer_ids[j] > N) return fail(CBW_ERR_INVALID, "layer id out of range [0, n_layers]");
        max_id = std::max(max_id, (int)layer_ids[j]);
    }
    const int last_layer = (normalize & 2) ? std::min(max_id, N) : N;   // bit 1: stop after the last requested state
    hipStream_t st = (hipStream_t)stream;
    char* p = (char*)ws;
    float* hbuf = (float*)p; p += align_up((size_t)M * D * 4);
    uint16_t* x1 = (uint16_t*)p; p += align_up((size_t)B * 3000 * D * 2);
    uint16_t* a = (uint16_t*)p; p += align_up((size_t)M * D * 2);
    uint16_t* qkv = (uint16_t*)p; p += align_up((size_t)M * 3 * D * 2);
    uint16_t* att = (uint16_t*)p; p += align_up((size_t)M * D * 2);
    uint16_t* f = (uint16_t*)p; p += align_up((size_t)M * h->cfg.ffn_dim * 2);
    float* part = encoder_splitk_floats(h, B) > 0 ? (float*)p : nullptr;   // split-K partial sums
    auto capture = [&](int state) -> int {
        for (int j = 0; j < n_ids; ++j) {
            if (layer_ids[j] != state) continue;
            for (int b = 0; b < B; ++b)
                HIPCHK(hipMemcpyAsync(hs + (((size_t)b * n_ids + j) * T) * D, hbuf + (size_t)b * T * D,
                                      (size_t)T * D * 4, hipMemcpyDeviceToDevice, st));
        }
        return CBW_OK;
    };
    // conv1 (k3, p1) + GELU: [B][1][3000][cpad] -> [B][1][3000][D]
    {
        ConvArgs c{};
        c.x = mel; c.w = h->conv1.w.p; c.bias = h->conv1.b.as<float>(); c.y = x1; c.zero = h->zero.p;
        c.N = B; c.H = 1; c.W = 3000; c.Cin = h->cpad; c.Cout = D; c.KH = 1; c.KW = 3;
        c.sh = 1; c.sw = 1; c.ph = 0; c.pw = 1; c.Ho = 1; c.Wo = 3000; c.M = B * 3000; c.res_ld = c.y_ld = D;
        c.flags = CBW_EPI_GELU;
        HIPCHK(cbw_conv_igemm(c, st));
    }
    // conv2 (k3, s2, p1) + GELU + positions (per clip: the position table is [1500][D])
    for (int b = 0; b < B; ++b) {
        ConvArgs c{};
        c.x = x1 + (size_t)b * 3000 * D; c.w = h->conv2.w.p; c.bias = h->conv2.b.as<float>(); c.res = h->pos.p;
        c.y = hbuf + (size_t)b * T * D; c.zero = h->zero.p;
        c.N = 1; c.H = 1; c.W = 3000; c.Cin = D; c.Cout = D; c.KH = 1; c.KW = 3;
        c.sh = 1; c.sw = 2; c.ph = 0; c.pw = 1; c.Ho = 1; c.Wo = T; c.M = T; c.res_ld = c.y_ld = D;
        c.flags = CBW_EPI_GELU | CBW_EPI_RES_F32 | CBW_EPI_OUT_F32 | CBW_EPI_RES_AFTER_ACT;
        HIPCHK(cbw_conv_igemm(c, st));
    }
    CHK(capture(0));
    for (int i = 0; i < last_layer && i < N; ++i) {
        auto& L = h->layers[i];
        HIPCHK(cbw_layernorm(hbuf, L.ln1_g.as<float>(), L.ln1_b.as<float>(), a, nullptr, M, D, 1e-5f, st));
        CHK(launch_conv(L.qkv, a, 1, 1, M, qkv, nullptr, 0, h->zero.p, st));
        HIPCHK(cbw_attention(qkv, att, B, T, H, 64, st));
        CHK(launch_conv(L.out, att, 1, 1, M, hbuf, hbuf, CBW_EPI_RES_F32 | CBW_EPI_OUT_F32, h->zero.p, st, nullptr,
                        nullptr, nullptr, nullptr, part));
        HIPCHK(cbw_layernorm(hbuf, L.ln2_g.as<float>(), L.ln2_b.as<float>(), a, nullptr, M, D, 1e-5f, st));
        CHK(launch_conv(L.fc1, a, 1, 1, M, f, nullptr, CBW_EPI_GELU, h->zero.p, st));
        CHK(launch_conv(L.fc2, f, 1, 1, M, hbuf, hbuf, CBW_EPI_RES_F32 | CBW_EPI_OUT_F32, h->zero.p, st, nullptr,
                        nullptr, nullptr, nullptr, part));
        if (i + 1 < N) CHK(capture(i + 1));
    }
    if (last_layer >= N) {
        for (int j = 0; j < n_ids; ++j) {
            if (layer_ids[j] != N) continue;
            for (int b = 0; b < B; ++b)
                HIPCHK(cbw_layernorm(hbuf + (size_t)b * T * D, h->lnf_g.as<float>(), h->lnf_b.as<float>(), nullptr,
                                     hs + (((size_t)b * n_ids + j) * T) * D, T, D, 1e-5f, st));
        }
    }
    if (normalize & 1) HIPCHK(cbw_l2norm_rows_f32(hs, (int64_t)B * n_ids * T, D, st));
    return CBW_OK;
}

// ------------------------------------------------------------------ decoder
}  // extern "C"

struct cbw_decoder {
    cbw_decoder_config cfg{};
    ParamStore ps;
    bool finalized = false;
    int Vpad = 0;
    DevBuf zero;
    DevBuf emb, pos;
    struct Layer {
        DevBuf ln1_g, ln1_b, ln2_g, ln2_b, ln3_g, ln3_b;
        ConvW qkv, out, cq, ck, cv, co, fc1, fc2;
    };
    std::vector<Layer> layers;
    DevBuf lnf_g, lnf_b;
};

namespace {
struct DecState {
    uint16_t *ks, *vs, *kc, *vc, *a, *qkv, *att, *qc, *f, *scratch, *enc;
    float* h;
    // prefill activations (max_len rows): residual stream, LN out, qkv, attention out, cross q, fc1 out
    float* ph;
    uint16_t *pa, *pqkv, *patt, *pqc, *pf;
    float* apart;   // split-key attention partials
    char* end;
};
bool dec_fuse_enabled() {   // CBW_DEC_FUSE=0 keeps the step's LayerNorms and K/V append as separate launches (A/B)
    const char* e = getenv("CBW_DEC_FUSE");
    return !(e && atoi(e) == 0);
}
bool dec_split_enabled() {   // CBW_DEC_SPLIT=0 runs the step's attention on the one-workgroup-per-row kernel (A/B)
    const char* e = getenv("CBW_DEC_SPLIT");
    return !(e && atoi(e) == 0);
}
bool dec_gemv_enabled(int B) {   // CBW_DEC_GEMV=0 runs the decode-step Linears on the tile kernels (A/B)
    const char* e = getenv("CBW_DEC_GEMV");
    return B <= 16 && !(e && atoi(e) == 0);
}

DecState dec_carve(const cbw_decoder* h, void* state, int B, int Benc) {
    const size_t L = h->cfg.n_layers, D = h->cfg.d_model, F = h->cfg.ffn_dim, ML = h->cfg.max_len;
    char* p = (char*)state;
    DecState s;
    s.ks = (uint16_t*)p; p += align_up(L * B * ML * D * 2);
    s.vs = (uint16_t*)p; p += align_up(L * B * ML * D * 2);
    s.kc = (uint16_t*)p; p += align_up(L * Benc * 1500 * D * 2);
    s.vc = (uint16_t*)p; p += align_up(L * Benc * 1500 * D * 2);
    s.h = (float*)p; p += align_up((size_t)B * D * 4);
    s.a = (uint16_t*)p; p += align_up((size_t)B * D * 2);
    s.qkv = (uint16_t*)p; p += align_up((size_t)B * 3 * D * 2);
    s.att = (uint16_t*)p; p += align_up((size_t)B * D * 2);
    s.qc = (uint16_t*)p; p += align_up((size_t)B * D * 2);
    s.f = (uint16_t*)p; p += align_up((size_t)B * F * 2);
    s.scratch = (uint16_t*)p; p += align_up((size_t)B * ML * D * 2);
    s.enc = (uint16_t*)p; p += align_up((size_t)Benc * 1500 * D * 2);
    s.ph = (float*)p; p += align_up(ML * D * 4);
    s.pa = (uint16_t*)p; p += align_up(ML * D * 2);
    s.pqkv = (uint16_t*)p; p += align_up(ML * 3 * D * 2);
    s.patt = (uint16_t*)p; p += align_up(ML * D * 2);
    s.pqc = (uint16_t*)p; p += align_up(ML * D * 2);
    s.pf = (uint16_t*)p; p += align_up(ML * F * 2);
    s.apart = (float*)p; p += align_up((size_t)cbw_dec_attn_split_floats(B, h->cfg.n_heads) * 4);
    s.end = p;
    return s;
}
int64_t dec_state_bytes(const cbw_decoder* h, int B, int Benc) {   // the carve of a state at address 0
    return (int64_t)(dec_carve(h, nullptr, B, Benc).end - (char*)nullptr);
}
// the step's attention: split-key kernel (K/V read once per kv batch) when it applies, else one workgroup per row
int dec_self_split_keys() {   // CBW_DEC_SELF_SPLIT=N: self-attention over more than N keys on the split kernel
    const char* e = getenv("CBW_DEC_SELF_SPLIT");
    return e ? atoi(e) : 0;
}
bool dec_self_one_launch() {   // CBW_DEC_SELF_ONE=0: self-attention on the split kernel + combine (A/B)
    const char* e = getenv("CBW_DEC_SELF_ONE");
    return !(e && atoi(e) == 0);
}
hipError_t dec_attend(const DecState& s, const uint16_t* q, int ldq, const uint16_t* kc, const uint16_t* vc,
                      int64_t kv_bstride, int n_keys, int rows_per_kv, uint16_t* out, int B, int H, int D,
                      hipStream_t st, const int* n_keys_pos = nullptr, bool self = false, int nk_rows = 0) {
    if (self && rows_per_kv == 1 && n_keys <= 448 && dec_split_enabled() && dec_self_one_launch())
        return cbw_dec_self_attn(q, ldq, kc, vc, kv_bstride, n_keys, out, B, H, D, st, n_keys_pos, nk_rows);
    if (self && !n_keys_pos && n_keys <= dec_self_split_keys())
        return cbw_dec_attention(q, ldq, kc, vc, kv_bstride, n_keys, rows_per_kv, out, B, H, D, st);
    if (n_keys_pos || (dec_split_enabled() && rows_per_kv <= 8))
        return cbw_dec_attn_split(q, ldq, kc, vc, kv_bstride, n_keys, rows_per_kv, out, B, H, D, s.apart, st,
                                  n_keys_pos, nk_rows);
    return cbw_dec_attention(q, ldq, kc, vc, kv_bstride, n_keys, rows_per_kv, out, B, H, D, st);
}
}  // namespace

extern "C" {

int cbw_decoder_create(const cbw_decoder_config* cfg, cbw_decoder** out) {
    if (!cfg || !out) return fail(CBW_ERR_INVALID, "null argument");
    if (cfg->n_heads < 1 || cfg->d_model % 128 || cfg->d_model / cfg->n_heads != 64 || cfg->ffn_dim % 128 ||
        cfg->n_layers < 1 || cfg->vocab < 2 || cfg->max_len < 1 || cfg->max_len > 448)
        return fail(CBW_ERR_INVALID, "decoder needs d_model % 128 == 0, head_dim 64, ffn_dim % 128 == 0, max_len <= 448");
    auto h = std::make_unique<cbw_decoder>();
    h->cfg = *cfg;
    h->Vpad = (cfg->vocab + 127) / 128 * 128;
    CHK(h->zero.alloc(256));
    HIPCHK(hipMemset(h->zero.p, 0, 256));
    *out = h.release();
    return CBW_OK;
}

int cbw_decoder_destroy(cbw_decoder* h) {
    delete h;
    return CBW_OK;
}

int cbw_decoder_set_param(cbw_decoder* h, const char* name, const float* host, int64_t numel) {
    if (!h) return fail(CBW_ERR_INVALID, "null handle");
    h->finalized = false;
    return h->ps.set(name, host, numel);
}

int cbw_decoder_vocab_padded(cbw_decoder* h) { return h ? h->Vpad : -1; }

int cbw_decoder_finalize(cbw_decoder* h) {
    if (!h) return fail(CBW_ERR_INVALID, "null handle");
    const int D = h->cfg.d_model, F = h->cfg.ffn_dim, V = h->cfg.vocab;
    int rc;
    {
        const auto* e = h->ps.get("embed_tokens.weight", (size_t)V * D, &rc);
        if (!e) return rc;
        std::vector<float> ep((size_t)h->Vpad * D, 0.f);
        std::copy(e->begin(), e->end(), ep.begin());
        CHK(h->emb.upload(to_bf16(ep)));
        const auto* p = h->ps.get("embed_positions.weight", (size_t)448 * D, &rc);
        if (!p) return rc;
        CHK(h->pos.upload(*p));
    }
    const float qscale = 1.0f / std::sqrt(64.0f);
    h->layers.clear();
    h->layers.resize(h->cfg.n_layers);
    for (int i = 0; i < h->cfg.n_layers; ++i) {
        auto& L = h->layers[i];
        const std::string p = "layers." + std::to_string(i);
        CHK(upload_vec(h->ps, p + ".self_attn_layer_norm.weight", D, L.ln1_g));
        CHK(upload_vec(h->ps, p + ".self_attn_layer_norm.bias", D, L.ln1_b));
        CHK(upload_vec(h->ps, p + ".encoder_attn_layer_norm.weight", D, L.ln2_g));
        CHK(upload_vec(h->ps, p + ".encoder_attn_layer_norm.bias", D, L.ln2_b));
        CHK(upload_vec(h->ps, p + ".final_layer_norm.weight", D, L.ln3_g));
        CHK(upload_vec(h->ps, p + ".final_layer_norm.bias", D, L.ln3_b));
        {
            const auto* wq = h->ps.get(p + ".self_attn.q_proj.weight", (size_t)D * D, &rc); if (!wq) return rc;
            const auto* wk = h->ps.get(p + ".self_attn.k_proj.weight", (size_t)D * D, &rc); if (!wk) return rc;
            const auto* wv = h->ps.get(p + ".self_attn.v_proj.weight", (size_t)D * D, &rc); if (!wv) return rc;
            const auto* bq = h->ps.get(p + ".self_attn.q_proj.bias", D, &rc); if (!bq) return rc;
            const auto* bv = h->ps.get(p + ".self_attn.v_proj.bias", D, &rc); if (!bv) return rc;
            std::vector<float> w((size_t)3 * D * D), b((size_t)3 * D, 0.f);
            for (size_t j = 0; j < (size_t)D * D; ++j) {
                w[j] = (*wq)[j] * qscale;
                w[(size_t)D * D + j] = (*wk)[j];
                w[(size_t)2 * D * D + j] = (*wv)[j];
            }
            for (int j = 0; j < D; ++j) { b[j] = (*bq)[j] * qscale; b[2 * D + j] = (*bv)[j]; }
            L.qkv.cin = D; L.qkv.cout = 3 * D; L.qkv.k = 1;
            CHK(L.qkv.w.upload(to_bf16(w)));
            CHK(L.qkv.b.upload(b));
        }
        CHK(upload_linear(h->ps, p + ".self_attn.out_proj", D, D, true, L.out));
        CHK(upload_linear(h->ps, p + ".encoder_attn.q_proj", D, D, true, L.cq, qscale));
        CHK(upload_linear(h->ps, p + ".encoder_attn.k_proj", D, D, false, L.ck));
        CHK(upload_linear(h->ps, p + ".encoder_attn.v_proj", D, D, true, L.cv));
        CHK(upload_linear(h->ps, p + ".encoder_attn.out_proj", D, D, true, L.co));
        CHK(upload_linear(h->ps, p + ".fc1", F, D, true, L.fc1));
        CHK(upload_linear(h->ps, p + ".fc2", D, F, true, L.fc2));
    }
    CHK(upload_vec(h->ps, "layer_norm.weight", D, h->lnf_g));
    CHK(upload_vec(h->ps, "layer_norm.bias", D, h->lnf_b));
    h->finalized = true;
    return CBW_OK;
}

int64_t cbw_decoder_state_bytes(cbw_decoder* h, int B, int Benc) {
    if (!h || B <= 0 || Benc <= 0 || B % Benc) return -1;
    return dec_state_bytes(h, B, Benc);
}

int cbw_decoder_cross_kv(cbw_decoder* h, const float* enc_out, int Benc, void* state, int64_t state_bytes, int B,
                         cbw_stream_t stream) {
    if (!h || !enc_out || !state) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized) return fail(CBW_ERR_STATE, "cbw_decoder_finalize not called");
    if (B <= 0 || Benc <= 0 || B % Benc) return fail(CBW_ERR_INVALID, "B must be a positive multiple of Benc");
    if (state_bytes < dec_state_bytes(h, B, Benc)) return fail(CBW_ERR_OOM, "decoder state too small");
    hipStream_t st = (hipStream_t)stream;
    const int D = h->cfg.d_model;
    DecState s = dec_carve(h, state, B, Benc);
    HIPCHK(cbw_cast_permute_lbtd(enc_out, s.enc, 1, 1, Benc * 1500, D, st));
    const size_t per = (size_t)Benc * 1500 * D;
    for (int l = 0; l < h->cfg.n_layers; ++l) {
        CHK(launch_conv(h->layers[l].ck, s.enc, 1, 1, Benc * 1500, s.kc + l * per, nullptr, 0, h->zero.p, st));
        CHK(launch_conv(h->layers[l].cv, s.enc, 1, 1, Benc * 1500, s.vc + l * per, nullptr, 0, h->zero.p, st));
    }
    return CBW_OK;
}

int cbw_decoder_cross_kv_slot(cbw_decoder* h, const float* enc_out, int slot, int Benc, void* state,
                              int64_t state_bytes, int B, cbw_stream_t stream) {
    if (!h || !enc_out || !state) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized) return fail(CBW_ERR_STATE, "cbw_decoder_finalize not called");
    if (B <= 0 || Benc <= 0 || B % Benc || slot < 0 || slot >= Benc)
        return fail(CBW_ERR_INVALID, "B must be a positive multiple of Benc, 0 <= slot < Benc");
    if (state_bytes < dec_state_bytes(h, B, Benc)) return fail(CBW_ERR_OOM, "decoder state too small");
    hipStream_t st = (hipStream_t)stream;
    const int D = h->cfg.d_model;
    DecState s = dec_carve(h, state, B, Benc);
    const size_t per = (size_t)Benc * 1500 * D, at = (size_t)slot * 1500 * D;
    HIPCHK(cbw_cast_permute_lbtd(enc_out, s.enc + at, 1, 1, 1500, D, st));
    for (int l = 0; l < h->cfg.n_layers; ++l) {
        CHK(launch_conv(h->layers[l].ck, s.enc + at, 1, 1, 1500, s.kc + l * per + at, nullptr, 0, h->zero.p, st));
        CHK(launch_conv(h->layers[l].cv, s.enc + at, 1, 1, 1500, s.vc + l * per + at, nullptr, 0, h->zero.p, st));
    }
    return CBW_OK;
}

}  // extern "C"
namespace {
// one decode step; pos_dev (optional) = the position read on the device (pos is then unused): every launch
// argument is then independent of the position, so the step can be captured once and replayed.  pos_rows: pos_dev
// holds one position per row (the rows of several windows, each at its own position, in one step)
int dec_step(cbw_decoder* h, const int32_t* tokens, int pos, const int32_t* pos_dev, int B, int Benc, void* state,
             int64_t state_bytes, float* logits, cbw_stream_t stream, int pos_rows = 0) {
    if (!h || !tokens || !state || !logits) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized) return fail(CBW_ERR_STATE, "cbw_decoder_finalize not called");
    if (B <= 0 || Benc <= 0 || B % Benc || (!pos_dev && (pos < 0 || pos >= h->cfg.max_len)))
        return fail(CBW_ERR_INVALID, "bad B/Benc/pos");
    if (state_bytes < dec_state_bytes(h, B, Benc)) return fail(CBW_ERR_OOM, "decoder state too small");
    hipStream_t st = (hipStream_t)stream;
    const int D = h->cfg.d_model, H = h->cfg.n_heads, ML = h->cfg.max_len;
    DecState s = dec_carve(h, state, B, Benc);
    // the step's Linears: skinny GEMV (gemv.hip) for <= 16 rows, else the implicit-GEMM tiles
    const bool gemv = dec_gemv_enabled(B);
    auto lin = [&](const ConvW& c, const void* x, void* y, const void* res, int flags) -> int {
        if (!gemv) return launch_conv(c, x, 1, 1, B, y, res, flags, h->zero.p, st);
        GemvArgs g{};
        g.x = (const bf16*)x; g.ldx = c.cin; g.w = c.w.as<bf16>(); g.bias = c.b.as<float>();
        g.res = res; g.res_ld = c.cout; g.y = y; g.ldy = c.cout;
        g.M = B; g.N = c.cout; g.K = c.cin; g.flags = flags | (c.relu ? CBW_EPI_RELU : 0);
        HIPCHK(cbw_gemv(g, st));
        return CBW_OK;
    };
    // LayerNorm -> Linear pairs: on the GEMV the LayerNorm runs in its prologue (and the qkv projection
    // appends K/V to the cache in its epilogue), else as separate launches
    const bool fuse = gemv && dec_fuse_enabled() && cbw_gemv_ln_ok(B, D);
    if (pos_dev && !fuse)
        return fail(CBW_ERR_INVALID, "device-position steps need the fused GEMV path (<= 16 rows, CBW_DEC_GEMV / "
                                     "CBW_DEC_FUSE on)");
    auto ln_lin = [&](const DevBuf& g, const DevBuf& b, const ConvW& c, void* y, int flags, uint16_t* kk,
                      uint16_t* vv) -> int {
        if (!fuse) {
            HIPCHK(cbw_layernorm(s.h, g.as<float>(), b.as<float>(), s.a, nullptr, B, D, 1e-5f, st));
            CHK(lin(c, s.a, y, nullptr, flags));
            if (kk) HIPCHK(cbw_dec_kv_append((const uint16_t*)y, kk, vv, B, D, ML, pos, st));
            return CBW_OK;
        }
        GemvArgs a{};
        a.xf = s.h; a.ldx = D; a.ln_g = g.as<float>(); a.ln_b = b.as<float>(); a.ln_eps = 1e-5f;
        a.w = c.w.as<bf16>(); a.bias = c.b.as<float>(); a.y = y; a.ldy = c.cout;
        a.M = B; a.N = c.cout; a.K = c.cin; a.flags = flags | (c.relu ? CBW_EPI_RELU : 0);
        if (kk) {
            a.kv_k = (bf16*)kk + (pos_dev ? 0 : (size_t)pos * D); a.kv_v = (bf16*)vv + (pos_dev ? 0 : (size_t)pos * D);
            a.kv_ld = (int64_t)ML * D; a.kv_D = D; a.kv_pos = pos_dev; a.kv_pos_rows = pos_rows;
        }
        HIPCHK(cbw_gemv(a, st));
        return CBW_OK;
    };
    HIPCHK(cbw_dec_embed(tokens, h->emb.as<uint16_t>(), h->pos.as<float>(), pos, s.h, B, D, st, 0, pos_dev, pos_rows));
    const size_t self_per = (size_t)B * ML * D, cross_per = (size_t)Benc * 1500 * D;
    for (int l = 0; l < h->cfg.n_layers; ++l) {
        auto& L = h->layers[l];
        uint16_t* kl = s.ks + l * self_per;
        uint16_t* vl = s.vs + l * self_per;
        CHK(ln_lin(L.ln1_g, L.ln1_b, L.qkv, s.qkv, 0, kl, vl));
        HIPCHK(dec_attend(s, s.qkv, 3 * D, kl, vl, (int64_t)ML * D, pos_dev ? ML : pos + 1, 1, s.att, B, H, D, st,
                          pos_dev, true, pos_rows));
        CHK(lin(L.out, s.att, s.h, s.h, CBW_EPI_RES_F32 | CBW_EPI_OUT_F32));
        CHK(ln_lin(L.ln2_g, L.ln2_b, L.cq, s.qc, 0, nullptr, nullptr));
        HIPCHK(dec_attend(s, s.qc, D, s.kc + l * cross_per, s.vc + l * cross_per, (int64_t)1500 * D, 1500, B / Benc,
                          s.att, B, H, D, st));
        CHK(lin(L.co, s.att, s.h, s.h, CBW_EPI_RES_F32 | CBW_EPI_OUT_F32));
        CHK(ln_lin(L.ln3_g, L.ln3_b, L.fc1, s.f, CBW_EPI_GELU, nullptr, nullptr));
        CHK(lin(L.fc2, s.f, s.h, s.h, CBW_EPI_RES_F32 | CBW_EPI_OUT_F32));
    }
    if (fuse) {   // final LayerNorm in the vocabulary projection's prologue
        GemvArgs g{};
        g.xf = s.h; g.ldx = D; g.ln_g = h->lnf_g.as<float>(); g.ln_b = h->lnf_b.as<float>(); g.ln_eps = 1e-5f;
        g.w = h->emb.as<bf16>(); g.y = logits; g.ldy = h->Vpad;
        g.M = B; g.N = h->Vpad; g.K = D; g.flags = CBW_EPI_OUT_F32;
        HIPCHK(cbw_gemv(g, st));
        return CBW_OK;
    }
    HIPCHK(cbw_layernorm(s.h, h->lnf_g.as<float>(), h->lnf_b.as<float>(), s.a, nullptr, B, D, 1e-5f, st));
    ConvArgs c{};
    c.x = s.a; c.w = h->emb.p; c.bias = nullptr; c.res = nullptr; c.y = logits; c.zero = h->zero.p;
    c.N = 1; c.H = 1; c.W = B; c.Cin = D; c.Cout = h->Vpad; c.KH = 1; c.KW = 1; c.sh = c.sw = 1; c.ph = c.pw = 0;
    c.Ho = 1; c.Wo = B; c.M = B; c.res_ld = c.y_ld = h->Vpad; c.flags = CBW_EPI_OUT_F32;
    if (gemv) {   // vocabulary projection
        GemvArgs g{};
        g.x = (const bf16*)s.a; g.ldx = D; g.w = h->emb.as<bf16>(); g.y = logits; g.ldy = h->Vpad;
        g.M = B; g.N = h->Vpad; g.K = D; g.flags = CBW_EPI_OUT_F32;
        HIPCHK(cbw_gemv(g, st));
    } else {
        HIPCHK(cbw_conv_igemm(c, st));
    }
    return CBW_OK;
}

}  // namespace
extern "C" {

int cbw_decoder_step(cbw_decoder* h, const int32_t* tokens, int pos, int B, int Benc, void* state, int64_t state_bytes,
                     float* logits, cbw_stream_t stream) {
    return dec_step(h, tokens, pos, nullptr, B, Benc, state, state_bytes, logits, stream);
}

int cbw_decoder_step_dev(cbw_decoder* h, const int32_t* tokens, const int32_t* pos_dev, int B, int Benc, void* state,
                         int64_t state_bytes, float* logits, cbw_stream_t stream) {
    if (!pos_dev) return fail(CBW_ERR_INVALID, "null pos_dev");
    return dec_step(h, tokens, 0, pos_dev, B, Benc, state, state_bytes, logits, stream);
}

int cbw_decoder_step_rows(cbw_decoder* h, const int32_t* tokens, const int32_t* pos_rows, int B, int Benc, void* state,
                          int64_t state_bytes, float* logits, cbw_stream_t stream) {
    if (!pos_rows) return fail(CBW_ERR_INVALID, "null pos_rows");
    return dec_step(h, tokens, 0, pos_rows, B, Benc, state, state_bytes, logits, stream, 1);
}

int cbw_decoder_prefill(cbw_decoder* h, const int32_t* tokens, int T, int B, int Benc, void* state,
                        int64_t state_bytes, float* logits, cbw_stream_t stream) {
    if (Benc != 1) return fail(CBW_ERR_INVALID, "prefill needs Benc == 1 (cbw_decoder_prefill_rows: one window of several)");
    return cbw_decoder_prefill_rows(h, tokens, T, 0, 0, B, B, Benc, state, state_bytes, logits, stream);
}

}  // extern "C"

namespace {
// The prefill layers: the T tokens as rows at positions 0..T-1, their K/V into cache rows [r0, r0 + nb) (attending to
// encoder slot `slot`); s.ph ends as the last layer's residual stream.  probes (n_probe > 0): right after layer l's
// cross-attention query, the probabilities of each listed (layer, head) pair of that layer -> probs[i] [T][1500].
int dec_prefill_layers(cbw_decoder* h, const int32_t* tokens, int T, int slot, int r0, int nb, int B, int Benc,
                       const DecState& s, hipStream_t st, const int32_t* probe = nullptr, int n_probe = 0,
                       float* probs = nullptr) {
    const int D = h->cfg.d_model, H = h->cfg.n_heads, ML = h->cfg.max_len;
    // the T prefix tokens as T rows at positions 0..T-1 (the beams are identical through a forced prefix:
    // one row set, its K/V replicated into every beam row of the cache: rows r0 .. r0 + nb - 1, which attend to
    // encoder slot `slot`)
    HIPCHK(cbw_dec_embed(tokens, h->emb.as<uint16_t>(), h->pos.as<float>(), 0, s.ph, T, D, st, 1));
    const size_t self_per = (size_t)B * ML * D, cross_per = (size_t)Benc * 1500 * D;
    for (int l = 0; l < h->cfg.n_layers; ++l) {
        auto& L = h->layers[l];
        uint16_t* kl = s.ks + l * self_per + (size_t)r0 * ML * D;
        uint16_t* vl = s.vs + l * self_per + (size_t)r0 * ML * D;
        HIPCHK(cbw_layernorm(s.ph, L.ln1_g.as<float>(), L.ln1_b.as<float>(), s.pa, nullptr, T, D, 1e-5f, st));
        CHK(launch_conv(L.qkv, s.pa, 1, 1, T, s.pqkv, nullptr, 0, h->zero.p, st));
        HIPCHK(cbw_dec_kv_prefill(s.pqkv, kl, vl, T, nb, D, ML, st));
        HIPCHK(cbw_dec_attention(s.pqkv, 3 * D, kl, vl, (int64_t)ML * D, T, T, s.patt, T, H, D, st, 1));
        CHK(launch_conv(L.out, s.patt, 1, 1, T, s.ph, s.ph, CBW_EPI_RES_F32 | CBW_EPI_OUT_F32, h->zero.p, st));
        HIPCHK(cbw_layernorm(s.ph, L.ln2_g.as<float>(), L.ln2_b.as<float>(), s.pa, nullptr, T, D, 1e-5f, st));
        CHK(launch_conv(L.cq, s.pa, 1, 1, T, s.pqc, nullptr, 0, h->zero.p, st));
        for (int i = 0; i < n_probe; ++i)
            if (probe[2 * i] == l)
                HIPCHK(cbw_dec_cross_probs(s.pqc, D, s.kc + l * cross_per + (size_t)slot * 1500 * D, 1500, T, D,
                                           probe[2 * i + 1], probs + (size_t)i * T * 1500, st));
        HIPCHK(cbw_dec_attention(s.pqc, D, s.kc + l * cross_per + (size_t)slot * 1500 * D,
                                 s.vc + l * cross_per + (size_t)slot * 1500 * D, (int64_t)1500 * D, 1500, T,
                                 s.patt, T, H, D, st));
        CHK(launch_conv(L.co, s.patt, 1, 1, T, s.ph, s.ph, CBW_EPI_RES_F32 | CBW_EPI_OUT_F32, h->zero.p, st));
        HIPCHK(cbw_layernorm(s.ph, L.ln3_g.as<float>(), L.ln3_b.as<float>(), s.pa, nullptr, T, D, 1e-5f, st));
        CHK(launch_conv(L.fc1, s.pa, 1, 1, T, s.pf, nullptr, CBW_EPI_GELU, h->zero.p, st));
        CHK(launch_conv(L.fc2, s.pf, 1, 1, T, s.ph, s.ph, CBW_EPI_RES_F32 | CBW_EPI_OUT_F32, h->zero.p, st));
    }
    return CBW_OK;
}
}  // namespace

extern "C" {

int cbw_decoder_prefill_rows(cbw_decoder* h, const int32_t* tokens, int T, int slot, int r0, int nb, int B, int Benc,
                             void* state, int64_t state_bytes, float* logits, cbw_stream_t stream) {
    if (!h || !tokens || !state || !logits) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized) return fail(CBW_ERR_STATE, "cbw_decoder_finalize not called");
    if (B < 1 || Benc < 1 || B % Benc || T < 1 || T > h->cfg.max_len || slot < 0 || slot >= Benc || nb < 1 || r0 < 0 ||
        r0 + nb > B)
        return fail(CBW_ERR_INVALID, "prefill needs 1 <= T <= max_len, 0 <= slot < Benc, rows [r0, r0 + nb) within B");
    if (state_bytes < dec_state_bytes(h, B, Benc)) return fail(CBW_ERR_OOM, "decoder state too small");
    hipStream_t st = (hipStream_t)stream;
    const int D = h->cfg.d_model;
    DecState s = dec_carve(h, state, B, Benc);
    CHK(dec_prefill_layers(h, tokens, T, slot, r0, nb, B, Benc, s, st));
    // logits of the last prefix token only
    const float* last = s.ph + (size_t)(T - 1) * D;
    HIPCHK(cbw_layernorm(last, h->lnf_g.as<float>(), h->lnf_b.as<float>(), s.pa, nullptr, 1, D, 1e-5f, st));
    if (dec_gemv_enabled(B)) {   // the vocabulary projection on the same kernel as the step's
        GemvArgs g{};
        g.x = (const bf16*)s.pa; g.ldx = D; g.w = h->emb.as<bf16>(); g.y = logits; g.ldy = h->Vpad;
        g.M = 1; g.N = h->Vpad; g.K = D; g.flags = CBW_EPI_OUT_F32;
        HIPCHK(cbw_gemv(g, st));
    } else {
        ConvArgs c{};
        c.x = s.pa; c.w = h->emb.p; c.y = logits; c.zero = h->zero.p;
        c.N = 1; c.H = 1; c.W = 1; c.Cin = D; c.Cout = h->Vpad; c.KH = 1; c.KW = 1; c.sh = c.sw = 1;
        c.Ho = 1; c.Wo = 1; c.M = 1; c.res_ld = c.y_ld = h->Vpad; c.flags = CBW_EPI_OUT_F32;
        HIPCHK(cbw_conv_igemm(c, st));
    }
    return CBW_OK;
}

int cbw_decoder_cross_attn_probs(cbw_decoder* h, const int32_t* tokens, int T, const int32_t* heads, int n, int B,
                                 int Benc, void* state, int64_t state_bytes, float* probs, cbw_stream_t stream) {
    if (!h || !tokens || !heads || !state || !probs) return fail(CBW_ERR_INVALID, "null argument");
    if (!h->finalized) return fail(CBW_ERR_STATE, "cbw_decoder_finalize not called");
    if (B < 1 || Benc < 1 || B % Benc || T < 1 || T > h->cfg.max_len || n < 1)
        return fail(CBW_ERR_INVALID, "cross_attn_probs needs 1 <= T <= max_len, n >= 1, B a multiple of Benc");
    if (h->cfg.d_model != 64 * h->cfg.n_heads) return fail(CBW_ERR_INVALID, "cross_attn_probs: head dim must be 64");
    for (int i = 0; i < n; ++i)
        if (heads[2 * i] < 0 || heads[2 * i] >= h->cfg.n_layers || heads[2 * i + 1] < 0 ||
            heads[2 * i + 1] >= h->cfg.n_heads)
            return fail(CBW_ERR_INVALID, "cross_attn_probs: (layer, head) out of range");
    if (state_bytes < dec_state_bytes(h, B, Benc)) return fail(CBW_ERR_OOM, "decoder state too small");
    DecState s = dec_carve(h, state, B, Benc);
    return dec_prefill_layers(h, tokens, T, 0, 0, 1, B, Benc, s, (hipStream_t)stream, heads, n, probs);
}

int cbw_dtw(const double* matrix, int rows, int cols, int32_t* text_idx, int32_t* time_idx, int* len) {
    if (!matrix || !text_idx || !time_idx || !len || rows < 1 || cols < 1) return fail(CBW_ERR_INVALID, "cbw_dtw: bad arguments");
    // transformers' _dynamic_time_warping, step for step: float32 cost and trace tables, each cost the f64 matrix entry
    // plus the chosen f32 predecessor rounded to f32 (numpy's float64 + float32 stored into a float32 array); strict
    // comparisons pick the diagonal, then the row above, else the column to the left
    const int R = rows + 1, C = cols + 1;
    std::vector<float> cost((size_t)R * C, std::numeric_limits<float>::infinity()), trace((size_t)R * C, -1.f);
    cost[0] = 0.f;
    for (int j = 1; j < C; ++j)
        for (int i = 1; i < R; ++i) {
            const float c0 = cost[(size_t)(i - 1) * C + j - 1], c1 = cost[(size_t)(i - 1) * C + j],
                        c2 = cost[(size_t)i * C + j - 1];
            float c, t;
            if (c0 < c1 && c0 < c2) c = c0, t = 0.f;
            else if (c1 < c0 && c1 < c2) c = c1, t = 1.f;
            else c = c2, t = 2.f;
            cost[(size_t)i * C + j] = (float)(matrix[(size_t)(i - 1) * cols + j - 1] + (double)c);
            trace[(size_t)i * C + j] = t;
        }
    for (int j = 0; j < C; ++j) trace[j] = 2.f;
    for (int i = 0; i < R; ++i) trace[(size_t)i * C] = 1.f;
    int i = rows, j = cols, n = 0;
    while (i > 0 || j > 0) {
        text_idx[n] = i - 1;
        time_idx[n] = j - 1;
        ++n;
        const float t = trace[(size_t)i * C + j];
        if (t == 0.f) --i, --j;
        else if (t == 1.f) --i;
        else if (t == 2.f) --j;
        else return fail(CBW_ERR_STATE, "cbw_dtw: unexpected trace entry");
    }
    std::reverse(text_idx, text_idx + n);
    std::reverse(time_idx, time_idx + n);
    *len = n;
    return CBW_OK;
}

int cbw_decoder_reorder(cbw_decoder* h, const int32_t* src_rows, int B, int Benc, int len, void* state,
                        int64_t state_bytes, cbw_stream_t stream) {
    if (!h || !src_rows || !state) return fail(CBW_ERR_INVALID, "null argument");
    if (B <= 0 || Benc <= 0 || B % Benc || len < 0 || len > h->cfg.max_len) return fail(CBW_ERR_INVALID, "bad arguments");
    if (state_bytes < dec_state_bytes(h, B, Benc)) return fail(CBW_ERR_OOM, "decoder state too small");
    if (len == 0) return CBW_OK;
    hipStream_t st = (hipStream_t)stream;
    const int D = h->cfg.d_model, ML = h->cfg.max_len;
    DecState s = dec_carve(h, state, B, Benc);
    const size_t self_per = (size_t)B * ML * D;
    if (B <= 16) {   // every layer's K and V in one in-place launch
        HIPCHK(cbw_dec_reorder_kv(s.ks, s.vs, src_rows, B, h->cfg.n_layers, (int64_t)self_per, (int64_t)ML * D,
                                  (int64_t)len * D, st));
        return CBW_OK;
    }
    for (int l = 0; l < h->cfg.n_layers; ++l) {
        for (uint16_t* cache : {s.ks + l * self_per, s.vs + l * self_per}) {
            HIPCHK(cbw_dec_gather_rows(cache, s.scratch, src_rows, B, (int64_t)ML * D, (int64_t)len * D, st));
            HIPCHK(hipMemcpy2DAsync(cache, (size_t)ML * D * 2, s.scratch, (size_t)ML * D * 2, (size_t)len * D * 2, B,
                                    hipMemcpyDeviceToDevice, st));
        }
    }
    return CBW_OK;
}

int cbw_logprob_topk(const float* logits, int B, int V, int ld, const float* bias, int64_t bias_ld, int k, float* lp,
                     int32_t* idx, cbw_stream_t stream) {
    if (!logits || !lp || !idx || B <= 0 || V <= 0 || ld < V || k < 1 || k > 16 || bias_ld < 0)
        return fail(CBW_ERR_INVALID, "bad arguments (k must be in [1, 16])");
    HIPCHK(cbw_logprob_topk_launch(logits, B, V, ld, bias, bias_ld, k, lp, idx, (hipStream_t)stream));
    return CBW_OK;
}

int cbw_beam_select(const float* lp, const int32_t* idx, int B, int k, int eos, double* beam_scores,
                    double* cand_score, int32_t* cand_row, int32_t* cand_tok, int32_t* tokens, int32_t* parents,
                    int32_t* ok, int32_t* ts_state, int32_t* st_out, int timestamp_begin, int count,
                    cbw_stream_t stream) {
    if (!lp || !idx || !beam_scores || !cand_score || !cand_row || !cand_tok || !tokens || !parents || !ok || !ts_state ||
        !st_out || B < 1 || B > 16 || k < 1 || k > 16)
        return fail(CBW_ERR_INVALID, "bad arguments (B and k in [1, 16])");
    HIPCHK(cbw_beam_select_launch(lp, idx, B, k, eos, beam_scores, cand_score, cand_row, cand_tok, tokens, parents, ok,
                                  ts_state, st_out, timestamp_begin, count, (hipStream_t)stream));
    return CBW_OK;
}
int cbw_timestamp_rules(const float* logits, int B, int V, int ld, const float* bias, const int32_t* state,
                        int timestamp_begin, int no_timestamps, int eos, int max_initial, float* bias_out,
                        cbw_stream_t stream) {
    if (!logits || !state || !bias_out || B <= 0 || V <= 0 || ld < V || timestamp_begin <= 0 ||
        timestamp_begin >= V || eos < 0 || eos >= V || no_timestamps < 0 || no_timestamps >= V)
        return fail(CBW_ERR_INVALID, "bad arguments");
    HIPCHK(cbw_timestamp_rules_launch(logits, B, V, ld, bias, state, timestamp_begin, no_timestamps, eos, max_initial,
                                      bias_out, (hipStream_t)stream));
    return CBW_OK;
}

// ------------------------------------------------------------------ building block
}  // extern "C"
namespace {
// 256 zero bytes per device (padding taps / rows past M of the building-block convs)
int block_zero_page(const void** out) {
    static thread_local std::map<int, std::shared_ptr<DevBuf>> zeros;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    auto it = zeros.find(dev);
    if (it == zeros.end()) {
        auto z = std::make_shared<DevBuf>();
        CHK(z->alloc(256));
        HIPCHK(hipMemset(z->p, 0, 256));
        it = zeros.emplace(dev, z).first;
    }
    *out = it->second->p;
    return CBW_OK;
}
}  // namespace
extern "C" {
int cbw_conv2d(const uint16_t* x, const uint16_t* w, const float* bias, const void* res, void* y, int N, int H, int W,
               int Cin, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int flags, cbw_stream_t stream) {
    if (!x || !w || !y || Cin % 64 || Cout % 64) return fail(CBW_ERR_INVALID, "cbw_conv2d: Cin and Cout must be multiples of 64");
    if (!((KH == 1 && KW == 1) || (KH == 3 && KW == 3) || (KH == 1 && KW == 3)))
        return fail(CBW_ERR_INVALID, "cbw_conv2d: kernel must be 1x1, 3x3 or 1x3");
    const void* zp = nullptr;
    CHK(block_zero_page(&zp));
    ConvArgs a{};
    a.x = x; a.w = w; a.bias = bias; a.res = res; a.y = y; a.zero = zp;
    a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.KH = KH; a.KW = KW;
    a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw;
    a.Ho = (H + 2 * ph - KH) / sh + 1;
    a.Wo = (W + 2 * pw - KW) / sw + 1;
    a.M = N * a.Ho * a.Wo;
    a.res_ld = a.y_ld = Cout;
    a.flags = flags;
    HIPCHK(cbw_conv_igemm(a, (hipStream_t)stream));
    return CBW_OK;
}

int cbw_gemm_splitk_factor(int M, int K, int N) {
    if (M <= 0 || K <= 0 || N <= 0) return fail(CBW_ERR_INVALID, "cbw_gemm_splitk_factor: bad shape");
    ConvArgs a{};
    a.KH = a.KW = 1; a.Cin = K; a.Cout = N; a.M = M;
    return cbw_conv_splitk_factor(a);
}

int cbw_encoder_attention(const uint16_t* qkv, uint16_t* out, int B, int T, int H, cbw_stream_t stream) {
    if (!qkv || !out || B <= 0 || T <= 0 || H <= 0) return fail(CBW_ERR_INVALID, "cbw_encoder_attention: bad argument");
    HIPCHK(cbw_attention(qkv, out, B, T, H, 64, (hipStream_t)stream));
    return CBW_OK;
}

int cbw_gemm(const uint16_t* x, const uint16_t* w, const float* bias, const void* res, void* y, int M, int K, int N,
             int flags, int ksplit, float* partial, int64_t partial_floats, cbw_stream_t stream) {
    if (!x || !w || !y || M <= 0 || K % 64 || N % 64 || ksplit < 0)
        return fail(CBW_ERR_INVALID, "cbw_gemm: K and N must be multiples of 64");
    const void* zp = nullptr;
    CHK(block_zero_page(&zp));
    ConvArgs a{};
    a.x = x; a.w = w; a.bias = bias; a.res = res; a.y = y; a.zero = zp;
    a.N = 1; a.H = 1; a.W = M; a.Cin = K; a.Cout = N; a.KH = a.KW = 1;
    a.sh = a.sw = 1; a.ph = a.pw = 0; a.Ho = 1; a.Wo = M; a.M = M;
    a.res_ld = a.y_ld = N;
    a.flags = flags;
    const int S = ksplit == 0 ? cbw_conv_splitk_factor(a) : ksplit;
    if (S > 1) {
        if (!partial || partial_floats < (int64_t)S * M * N) return fail(CBW_ERR_OOM, "cbw_gemm: partial buffer too small");
        if (N % 128 || S > K / 64) return fail(CBW_ERR_INVALID, "cbw_gemm: split-K needs N % 128 == 0 and S <= K / 64");
    }
    HIPCHK(cbw_conv_igemm_splitk(a, S, partial, (hipStream_t)stream));
    return CBW_OK;
}

int cbw_conv1x1_dual(const uint16_t* x, const uint16_t* x2, const uint16_t* w, const float* bias, const void* res,
                     void* y, int N, int H, int W, int Cin, int H2, int W2, int Cin2, int s2, int Cout, int flags,
                     cbw_stream_t stream) {
    if (!x || !x2 || !w || !y || N <= 0 || H <= 0 || W <= 0 || Cin % 64 || Cin2 % 64 || Cout % 128 || s2 < 1 ||
        (H - 1) * s2 >= H2 || (W - 1) * s2 >= W2 || (flags & ~1))
        return fail(CBW_ERR_INVALID, "cbw_conv1x1_dual: bad shapes");
    const void* zp = nullptr;
    CHK(block_zero_page(&zp));
    ConvArgs a{};
    a.x = x; a.w = w; a.bias = bias; a.res = res; a.y = y; a.zero = zp;
    a.x2 = x2; a.Cin2 = Cin2; a.H2 = H2; a.W2 = W2; a.s2 = s2;
    a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.KH = a.KW = 1;
    a.sh = a.sw = 1; a.ph = a.pw = 0;
    a.Ho = H; a.Wo = W;
    a.M = N * H * W;
    a.res_ld = a.y_ld = Cout;
    a.flags = flags;
    HIPCHK(cbw_conv_igemm(a, (hipStream_t)stream));
    return CBW_OK;
}

}  // extern "C"
