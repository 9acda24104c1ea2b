// Fused ResNet-50 stage-1 bottleneck block for gfx950: reduce 1x1 (256 -> 64) + BN + ReLU,
// 3x3 (64 -> 64) + BN + ReLU, expand 1x1 (64 -> 256) + BN, identity residual, ReLU -- one
// persistent launch; the two 64-channel intermediates never leave LDS.  A second kernel
// (bottleneck_s1_first_kernel, below) runs the stage's first block the same way.
//
// Reference: HF ResNetBottleNeckLayer (shortcut = identity when in == out channels and stride 1)
// as instantiated by efficient_kws/resnet.py:22-38 and run by Resnet.forward (resnet.py:51-58):
// stage 1 layers 1 and 2.  The unfused path (three conv_igemm launches) moves 7.3 MB per pair
// through HBM per block at LEF sizes; this kernel reads the block input once (+ halo columns)
// and writes the block output once.
//
// Work unit: one pair x TH (19) output rows x TW (6) output columns.  One 512-thread workgroup
// per CU (two waves per SIMD) walks a contiguous range of tiles; consecutive column tiles share
// their halo columns, which the previous tile has just pulled into L2, so HBM sees the block
// input about once.  LDS: the tile's input window X (168 px x 256 ch, 512-byte rows, 16-byte
// chunk index ^ (row & 15)), Wr (same layout), T1 (halo window x 64 ch) and T2 (tile x 64 ch)
// (144-byte pixel pitch), biases.  Each wave keeps its Wm / We slices in registers (88 VGPRs,
// loaded once).  Per tile:
//   phase R  T1 = relu(X . Wr + br), 0 outside the image (the 3x3's zero padding);
//            wave (mq, nh): 32 channels x 3 pixel fragments (5 LDS reads per 6 MFMAs; the (half,
//            quarter) split of phase M needed 7: 0.70 -> 0.67 ms per block at 500 pairs).  The residual the wave adds in
//            phase E is copied from X to registers; then the NEXT tile's window is issued into
//            X by glds and lands while phases M and E compute.
//   phase M  T2 = relu(conv3x3(T1) . Wm + bm); wave (mh, nq): 16 channels x 4 fragments.
//   phase E  y = relu(T2 . We + be + x); wave w: 32 channels x 8 fragments (two passes).
// y leaves by raw buffer stores (out-of-tile lanes dropped by the descriptor's range check), so
// every wave issues 16 per tile and the next tile's wait is vmcnt(16): the stores stay in flight.
// All MFMAs run transposed (C^T = W . X^T): a lane ends with 4 consecutive channels of one pixel.
//
// Measured (tools/bt_exp.sh, LEF chunk of 500 pairs): ~0.73 ms per block vs ~0.9 ms for the three
// separate convs; removing the MFMAs changes little, removing the window or the stores saves
// ~0.13 ms each -- the kernel is bound by in-core issue (LDS reads, address and epilogue VALU),
// not by HBM or MFMA.
#include "cbw_common.h"
#include "cbw_kernels.h"
#ifndef BT_EXP
#define BT_EXP 0   // diagnostic builds only (tools/bt_exp.sh): 1 no window refill, 2 no phase-M MFMAs,
                   // 3 no phase-R MFMAs, 4 no y stores
#endif

typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
// raw buffer store (LLVM intrinsic by asm label): lanes whose byte offset is past num_records are
// dropped by the hardware, so a wave issues the same number of stores for every tile (partial
// tiles included) and the top-of-tile wait can be a counted vmcnt that leaves them in flight.
__device__ void raw_buffer_store_v2i32(i32x2 vdata, i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.v2i32");

namespace {

constexpr int BT_TH = 19, BT_TW = 6;
constexpr int BT_CIN = 256, BT_MID = 64, BT_COUT = 256;
constexpr int BT_WW = BT_TW + 2;                   // halo window width
constexpr int BT_P1 = (BT_TH + 2) * BT_WW;         // 168 halo-window pixels
constexpr int BT_FR = ((BT_P1 + 15) / 16 + 3) / 4; // phase R fragments per pixel quarter: 3 (11 + a dummy)
constexpr int BT_P2 = BT_TH * BT_TW;               // 114 output pixels
constexpr int BT_F2 = (BT_P2 + 15) / 16;           // 8 fragments
constexpr int BT_FM = (BT_F2 + 1) / 2;             // phase M fragments per pixel half: 4
constexpr int BT_FE = (BT_F2 + 1) / 2;             // phase E fragments per half-pass: 4
constexpr int BT_PITCH = 144;                      // T1 / T2 bytes per pixel (64 ch + 16 pad)
constexpr int BT_X_BYTES = BT_P1 * 512;            // 86016: the tile's input window
constexpr int BT_WR = BT_X_BYTES;                  // Wr [64][256] bf16, 512-byte rows, swizzled like X
constexpr int BT_T1 = BT_WR + 64 * 512;            // + 32768
constexpr int BT_T2 = BT_T1 + BT_P1 * BT_PITCH;    // + 24192
constexpr int BT_BIAS = BT_T2 + BT_P2 * BT_PITCH;  // + 16416: biases br [64], bm [64], be [256] f32
constexpr int BT_LDS = BT_BIAS + (64 + 64 + 256) * 4;   // = 160928
static_assert(BT_LDS <= 163840, "LDS budget");
static_assert(2 * BT_FE * 2 == 16, "top-of-tile vmcnt assumes 16 y stores per wave");
constexpr int BT_XG = (BT_P1 + 15) / 16;           // window glds rounds (16 rows each; the last one partial)

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

CBW_DEV i32x4 buffer_rsrc(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    return i32x4{(int)(uint32_t)a, (int)(uint32_t)(a >> 32), (int)bytes, 0x00020000};
}

// An opaque 0 per tile: lane-dependent address terms built on it are recomputed inside the tile
// loop instead of being hoisted out of it into (spilled) registers.
CBW_DEV int launder_zero() {
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

CBW_DEV int x_off(int row, int chunk16) { return row * 512 + ((chunk16 ^ (row & 15)) << 4); }

__global__ __launch_bounds__(512, 1) void bottleneck_s1_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                               const bf16* __restrict__ wr, const float* __restrict__ br,
                                                               const bf16* __restrict__ wm, const float* __restrict__ bm,
                                                               const bf16* __restrict__ we, const float* __restrict__ be,
                                                               const void* __restrict__ zero, int N, int H, int W,
                                                               int nrt, int nct) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* X = smem;
    char* Wrs = smem + BT_WR;
    char* T1 = smem + BT_T1;
    char* T2 = smem + BT_T2;
    float* Bs = (float*)(smem + BT_BIAS);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int mh = wid >> 2, nq = wid & 3;     // phase M: pixel half x channel quarter
    const int mq = wid >> 1, nh = wid & 1;     // phase R: pixel quarter x channel half
    const int ntiles = N * nrt * nct;
    const int G = gridDim.x;

    // ---- once per workgroup: Wr and the biases -> LDS, this wave's Wm / We slices -> registers
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int e = k * 512 + tid;             // 16-byte chunk e of Wr: row e / 32, chunk e % 32
        const int row = e >> 5, c = e & 31;
        *(bf16x8*)(Wrs + x_off(row, c)) = *(const bf16x8*)(wr + row * BT_CIN + c * 8);
    }
    if (tid < 64) Bs[tid] = br[tid];
    else if (tid < 128) Bs[tid] = bm[tid - 64];
    if (tid < 256) Bs[128 + tid] = be[tid];
    bf16x8 wmf[18];                // Wm [64][3][3][64]: out ch 16 nq + fr, k-step (tap, half)
#pragma unroll
    for (int s = 0; s < 18; ++s) wmf[s] = *(const bf16x8*)(wm + (nq * 16 + fr) * 576 + s * 32 + fq * 8);
    bf16x8 wef[2][2];              // We [256][64]: out ch 32 w + 16 j + fr, k-step ks
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) wef[j][ks] = *(const bf16x8*)(we + (wid * 32 + j * 16 + fr) * BT_MID + ks * 32 + fq * 8);

    auto tile_origin = [&](int t, int& n, int& h0, int& w0) {
        n = t / (nrt * nct);
        const int rem = t - n * (nrt * nct);
        const int rt = rem / nct;
        h0 = rt * BT_TH;
        w0 = (rem - rt * nct) * BT_TW;
    };
    // the tile's input window -> X; wave-instruction g writes rows 16 g + 2 w, + 1 (lane / 32),
    // chunk lane % 32 (source chunk pre-swizzled, LDS destination linear)
    auto issue_window = [&](int t, int lz) {
        int n, h0, w0;
        tile_origin(t, n, h0, w0);
        const bf16* xn = x + (int64_t)n * H * W * BT_CIN;
        const int c = lane & 31;
#pragma unroll
        for (int g = 0; g < BT_XG; ++g) {
            if ((g * 16 + wid * 2) >= BT_P1) break;    // wave-uniform: rows past the window
            const int row = g * 16 + wid * 2 + (lane >> 5) + lz;
            const int i = row / BT_WW, jc = row - i * BT_WW;
            const int h = h0 - 1 + i, w = w0 - 1 + jc;
            const bool ok = h >= 0 && h < H && w >= 0 && w < W;
            const void* src = ok ? (const void*)(xn + ((int64_t)h * W + w) * BT_CIN + ((c ^ (row & 15)) * 8)) : zero;
            __builtin_amdgcn_global_load_lds(src, (void*)(X + (g * 16 + wid * 2) * 512), 16, 0, 0);
        }
    };

    // contiguous tile range per workgroup: consecutive column tiles share their halo columns,
    // which the previous tile has just pulled into L2
    const int per = (ntiles + G - 1) / G;
    const int t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
    if (t0 < t1) issue_window(t0, 0);
    for (int t = t0; t < t1; ++t) {
        int n, h0, w0;
        tile_origin(t, n, h0, w0);
        // this tile's window has landed (own DMAs; the previous tile's y stores drain too), every
        // other wave's as well, and every wave is done with the previous tile
        if (t == t0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // the previous tile's 16 y stores (2 x BT_FE x 2) stay in flight
        __builtin_amdgcn_s_barrier();
        const int frl = fr + launder_zero();

        // ---- phase R: wave (mq, nh) = fragments 3 mq .. 3 mq + 2 x channels 32 nh ..
        f32x4 ar[BT_FR][2];
#pragma unroll
        for (int i = 0; i < BT_FR; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) ar[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            bf16x8 bv[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) bv[j] = *(const bf16x8*)(Wrs + x_off(nh * 32 + j * 16 + frl, s * 4 + fq));
#pragma unroll
            for (int i = 0; i < BT_FR; ++i) {   // rows past the window read other LDS: discarded
                const bf16x8 av = *(const bf16x8*)(X + x_off((mq * BT_FR + i) * 16 + frl, s * 4 + fq));
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (BT_EXP != 3) ar[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv[j], av, ar[i][j], 0, 0, 0);
                    else asm volatile("" :: "v"(av), "v"(bv[j]));
                }
            }
        }
        // the residual this wave adds in phase E (channels 32 w + 16 j + 4 fq.., pixel 16 i + fr)
        u32x2 res[BT_F2][2];
#pragma unroll
        for (int i = 0; i < BT_F2; ++i) {
            const int q = min(i * 16 + frl, BT_P2 - 1);
            const int r = q / BT_TW, c = q - r * BT_TW;
            const int row = (r + 1) * BT_WW + (c + 1);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int ch = wid * 32 + j * 16 + fq * 4;
                res[i][j] = *(const u32x2*)(X + x_off(row, ch >> 3) + (ch & 7) * 2);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();              // X is free: the next window streams in during M and E
        if (BT_EXP != 1 && t + 1 < t1) issue_window(t + 1, frl - fr);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int ch = nh * 32 + j * 16 + fq * 4;
            const f32x4 brv = *(const f32x4*)(Bs + ch);
#pragma unroll
            for (int i = 0; i < BT_FR; ++i) {
                const int p = (mq * BT_FR + i) * 16 + frl;
                if (p >= BT_P1) continue;
                const int ii = p / BT_WW, jc = p - ii * BT_WW;
                const int h = h0 - 1 + ii, w = w0 - 1 + jc;
                const bool ok = h >= 0 && h < H && w >= 0 && w < W;
                bf16x4 o;
#pragma unroll
                for (int q = 0; q < 4; ++q) o[q] = f2bf(ok ? fmaxf(ar[i][j][q] + brv[q], 0.f) : 0.f);
                *(bf16x4*)(T1 + p * BT_PITCH + ch * 2) = o;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();

        // ---- phase M: wave (mh, nq) = fragments 4 mh .. 4 mh + 3 x channels 16 nq ..
        {
            f32x4 am[BT_FM];
            int pb[BT_FM];
            const int fb = mh * BT_FM;
#pragma unroll
            for (int i = 0; i < BT_FM; ++i) {
                am[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                const int q = min((fb + i) * 16 + frl, BT_P2 - 1);
                const int r = q / BT_TW, c = q - r * BT_TW;
                pb[i] = (r * BT_WW + c) * BT_PITCH + fq * 16;
            }
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int toff = ((tap / 3) * BT_WW + (tap % 3)) * BT_PITCH;
#pragma unroll
                for (int hh = 0; hh < 2; ++hh)
#pragma unroll
                    for (int i = 0; i < BT_FM; ++i) {   // (a fragment past the tile is a clamped dummy)
                        const bf16x8 av = *(const bf16x8*)(T1 + pb[i] + toff + hh * 64);
                        if (BT_EXP != 2) am[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wmf[tap * 2 + hh], av, am[i], 0, 0, 0);
                        else asm volatile("" :: "v"(av));
                    }
            }
            const int ch = nq * 16 + fq * 4;
            const f32x4 bmv = *(const f32x4*)(Bs + 64 + ch);
#pragma unroll
            for (int i = 0; i < BT_FM; ++i) {
                const int q = (fb + i) * 16 + frl;
                if (q >= BT_P2) continue;
                bf16x4 o;
#pragma unroll
                for (int k = 0; k < 4; ++k) o[k] = f2bf(fmaxf(am[i][k] + bmv[k], 0.f));
                *(bf16x4*)(T2 + q * BT_PITCH + ch * 2) = o;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();

        // ---- phase E: wave w = channels 32 w .., two passes of BT_FE fragments
        {
            const i32x4 yr = buffer_rsrc(y + (int64_t)n * H * W * BT_COUT, (uint32_t)H * W * BT_COUT * 2);
            f32x4 bev[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) bev[j] = *(const f32x4*)(Bs + 128 + wid * 32 + j * 16 + fq * 4);
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                f32x4 ae[BT_FE][2];
#pragma unroll
                for (int i = 0; i < BT_FE; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) ae[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                    for (int i = 0; i < BT_FE; ++i) {
                        const int q = min((half * BT_FE + i) * 16 + frl, BT_P2 - 1);
                        const bf16x8 av = *(const bf16x8*)(T2 + q * BT_PITCH + ks * 64 + fq * 16);
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            ae[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wef[j][ks], av, ae[i][j], 0, 0, 0);
                    }
#pragma unroll
                for (int i = 0; i < BT_FE; ++i) {
                    const int q = (half * BT_FE + i) * 16 + frl;
                    const int r = q / BT_TW, c = q - r * BT_TW;
                    const int h = h0 + r, w = w0 + c;
                    const bool ok = q < BT_P2 && h < H && w < W;
                    const int off = ok ? ((h * W + w) * BT_COUT + wid * 32 + fq * 4) * 2 : 0x7fffff00;
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        const bf16x4 rv = __builtin_bit_cast(bf16x4, res[half * BT_FE + i][j]);
                        bf16x4 o;
#pragma unroll
                        for (int k = 0; k < 4; ++k) o[k] = f2bf(fmaxf(ae[i][j][k] + bev[j][k] + bf2f(rv[k]), 0.f));
                        if (BT_EXP != 4) raw_buffer_store_v2i32(__builtin_bit_cast(i32x2, o), yr, off + j * 32, 0, 0);
                        else asm volatile("" :: "v"(o));
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------- the stage's first block (CIN 64)
// Same tiles and phases; the block input has 64 channels (128-byte window rows), there is no identity
// residual, and the projection shortcut 1x1 (64 -> 256) is folded into the expand as a second K-source:
// y = relu([T2 | x] . [We | Ws] + be + bs), we [256][128] (load_fused_expand_shortcut).  The window is
// double-buffered: the next tile's window lands during the whole current tile, and phase E reads the
// shortcut's centre pixels from the current one.
template <int CIN>
struct BtL {
    static constexpr int XROW = CIN * 2;                 // window bytes per pixel
    static constexpr int XC = CIN / 8;                   // 16-byte chunks per pixel
    static constexpr int SWM = XC >= 16 ? 15 : XC - 1;   // chunk swizzle mask
    static constexpr int NXB = CIN == 64 ? 2 : 1;        // window buffers
    static constexpr int X_BYTES = BT_P1 * XROW;         // 86016 / 21504
    static constexpr int WR = NXB * X_BYTES;             // Wr [64][CIN] bf16, swizzled like X
    static constexpr int T1 = WR + 64 * XROW;
    static constexpr int T2 = T1 + BT_P1 * BT_PITCH;     // + 24192
    static constexpr int BIAS = T2 + BT_P2 * BT_PITCH;   // + 16416: biases br [64], bm [64], be [256] f32
    static constexpr int LDS = BIAS + (64 + 64 + 256) * 4;   // 160928 / 93344
    static constexpr int RPI = 1024 / XROW;              // window rows per glds wave-instruction
    static constexpr int XG = (BT_P1 + 8 * RPI - 1) / (8 * RPI);   // window glds rounds
    static constexpr int KE = CIN == 64 ? 4 : 2;         // phase-E k-steps: T2 (+ the shortcut's x)
    static_assert(LDS <= 163840, "LDS budget");
    static_assert(BT_P1 % RPI == 0, "window rows per wave-instruction");
};
template <int CIN>
CBW_DEV int xw_off(int row, int chunk16) { return row * BtL<CIN>::XROW + ((chunk16 ^ (row & BtL<CIN>::SWM)) << 4); }

__global__ __launch_bounds__(512, 1) void bottleneck_s1_first_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                               const bf16* __restrict__ wr, const float* __restrict__ br,
                                                               const bf16* __restrict__ wm, const float* __restrict__ bm,
                                                               const bf16* __restrict__ we, const float* __restrict__ be,
                                                               const void* __restrict__ zero, int N, int H, int W,
                                                               int nrt, int nct) {
    constexpr int CIN = 64;
    using L = BtL<CIN>;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* const X0 = smem;
    char* Wrs = smem + L::WR;
    char* T1 = smem + L::T1;
    char* T2 = smem + L::T2;
    float* Bs = (float*)(smem + L::BIAS);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int mh = wid >> 2, nq = wid & 3;     // phase M: pixel half x channel quarter
    const int mq = wid >> 1, nh = wid & 1;     // phase R: pixel quarter x channel half
    const int ntiles = N * nrt * nct;
    const int G = gridDim.x;

    // ---- once per workgroup: Wr and the biases -> LDS, this wave's Wm / We slices -> registers
#pragma unroll
    for (int k = 0; k < 64 * L::XC / 512; ++k) {
        const int e = k * 512 + tid;             // 16-byte chunk e of Wr: row e / XC, chunk e % XC
        const int row = (unsigned)e / L::XC, c = e & (L::XC - 1);
        *(bf16x8*)(Wrs + xw_off<CIN>(row, c)) = *(const bf16x8*)(wr + row * CIN + c * 8);
    }
    if (tid < 64) Bs[tid] = br[tid];
    else if (tid < 128) Bs[tid] = bm[tid - 64];
    if (tid < 256) Bs[128 + tid] = be[tid];
    bf16x8 wmf[18];                // Wm [64][3][3][64]: out ch 16 nq + fr, k-step (tap, half)
#pragma unroll
    for (int s = 0; s < 18; ++s) wmf[s] = *(const bf16x8*)(wm + (nq * 16 + fr) * 576 + s * 32 + fq * 8);
    bf16x8 wef[2][L::KE];          // We [256][32 KE]: out ch 32 w + 16 j + fr, k-step ks
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < L::KE; ++ks)
            wef[j][ks] = *(const bf16x8*)(we + (wid * 32 + j * 16 + fr) * (32 * L::KE) + ks * 32 + fq * 8);

    auto tile_origin = [&](int t, int& n, int& h0, int& w0) {
        n = t / (nrt * nct);
        const int rem = t - n * (nrt * nct);
        const int rt = rem / nct;
        h0 = rt * BT_TH;
        w0 = (rem - rt * nct) * BT_TW;
    };
    // the tile's input window -> Xb; wave-instruction g writes rows RPI (8 g + w) .. + RPI - 1 (lane / XC),
    // chunk lane % XC (source chunk pre-swizzled, LDS destination linear)
    auto issue_window = [&](int t, int lz, char* Xb) {
        int n, h0, w0;
        tile_origin(t, n, h0, w0);
        const bf16* xn = x + (int64_t)n * H * W * CIN;
        const int c = lane & (L::XC - 1);
#pragma unroll
        for (int g = 0; g < L::XG; ++g) {
            const int r0 = (g * 8 + wid) * L::RPI;
            if (r0 >= BT_P1) break;                    // wave-uniform: rows past the window
            const int row = r0 + (int)((unsigned)lane / L::XC) + lz;
            const int i = row / BT_WW, jc = row - i * BT_WW;
            const int h = h0 - 1 + i, w = w0 - 1 + jc;
            const bool ok = h >= 0 && h < H && w >= 0 && w < W;
            const void* src = ok ? (const void*)(xn + ((int64_t)h * W + w) * CIN + ((c ^ (row & L::SWM)) * 8)) : zero;
            __builtin_amdgcn_global_load_lds(src, (void*)(Xb + r0 * L::XROW), 16, 0, 0);
        }
    };

    // contiguous tile range per workgroup: consecutive column tiles share their halo columns,
    // which the previous tile has just pulled into L2
    const int per = (ntiles + G - 1) / G;
    const int t0 = blockIdx.x * per, t1 = min(ntiles, t0 + per);
    if (t0 < t1) issue_window(t0, 0, X0);
    for (int t = t0; t < t1; ++t) {
        int n, h0, w0;
        tile_origin(t, n, h0, w0);
        char* const X = X0 + ((t - t0) & 1) * L::X_BYTES;   // this tile's window
        // this tile's window has landed (own DMAs; the previous tile's y stores drain too), every
        // other wave's as well, and every wave is done with the previous tile
        if (t == t0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // the previous tile's 16 y stores (2 x BT_FE x 2) stay in flight
        __builtin_amdgcn_s_barrier();
        const int frl = fr + launder_zero();
        // two window buffers: the next tile's window streams in during this whole tile (after the
        // 16 y stores, so the next top-of-tile vmcnt(16) still means "window landed")
        if (BT_EXP != 1 && t + 1 < t1) issue_window(t + 1, frl - fr, X0 + ((t - t0 + 1) & 1) * L::X_BYTES);

        // ---- phase R: wave (mq, nh) = fragments 3 mq .. 3 mq + 2 x channels 32 nh ..
        f32x4 ar[BT_FR][2];
#pragma unroll
        for (int i = 0; i < BT_FR; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) ar[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < L::XC / 4; ++s) {
            bf16x8 bv[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) bv[j] = *(const bf16x8*)(Wrs + xw_off<CIN>(nh * 32 + j * 16 + frl, s * 4 + fq));
#pragma unroll
            for (int i = 0; i < BT_FR; ++i) {   // rows past the window read other LDS: discarded
                const bf16x8 av = *(const bf16x8*)(X + xw_off<CIN>((mq * BT_FR + i) * 16 + frl, s * 4 + fq));
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    if (BT_EXP != 3) ar[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv[j], av, ar[i][j], 0, 0, 0);
                    else asm volatile("" :: "v"(av), "v"(bv[j]));
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int ch = nh * 32 + j * 16 + fq * 4;
            const f32x4 brv = *(const f32x4*)(Bs + ch);
#pragma unroll
            for (int i = 0; i < BT_FR; ++i) {
                const int p = (mq * BT_FR + i) * 16 + frl;
                if (p >= BT_P1) continue;
                const int ii = p / BT_WW, jc = p - ii * BT_WW;
                const int h = h0 - 1 + ii, w = w0 - 1 + jc;
                const bool ok = h >= 0 && h < H && w >= 0 && w < W;
                bf16x4 o;
#pragma unroll
                for (int q = 0; q < 4; ++q) o[q] = f2bf(ok ? fmaxf(ar[i][j][q] + brv[q], 0.f) : 0.f);
                *(bf16x4*)(T1 + p * BT_PITCH + ch * 2) = o;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();

        // ---- phase M: wave (mh, nq) = fragments 4 mh .. 4 mh + 3 x channels 16 nq ..
        {
            f32x4 am[BT_FM];
            int pb[BT_FM];
            const int fb = mh * BT_FM;
#pragma unroll
            for (int i = 0; i < BT_FM; ++i) {
                am[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                const int q = min((fb + i) * 16 + frl, BT_P2 - 1);
                const int r = q / BT_TW, c = q - r * BT_TW;
                pb[i] = (r * BT_WW + c) * BT_PITCH + fq * 16;
            }
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int toff = ((tap / 3) * BT_WW + (tap % 3)) * BT_PITCH;
#pragma unroll
                for (int hh = 0; hh < 2; ++hh)
#pragma unroll
                    for (int i = 0; i < BT_FM; ++i) {   // (a fragment past the tile is a clamped dummy)
                        const bf16x8 av = *(const bf16x8*)(T1 + pb[i] + toff + hh * 64);
                        if (BT_EXP != 2) am[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wmf[tap * 2 + hh], av, am[i], 0, 0, 0);
                        else asm volatile("" :: "v"(av));
                    }
            }
            const int ch = nq * 16 + fq * 4;
            const f32x4 bmv = *(const f32x4*)(Bs + 64 + ch);
#pragma unroll
            for (int i = 0; i < BT_FM; ++i) {
                const int q = (fb + i) * 16 + frl;
                if (q >= BT_P2) continue;
                bf16x4 o;
#pragma unroll
                for (int k = 0; k < 4; ++k) o[k] = f2bf(fmaxf(am[i][k] + bmv[k], 0.f));
                *(bf16x4*)(T2 + q * BT_PITCH + ch * 2) = o;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();

        // ---- phase E: wave w = channels 32 w .., two passes of BT_FE fragments
        {
            const i32x4 yr = buffer_rsrc(y + (int64_t)n * H * W * BT_COUT, (uint32_t)H * W * BT_COUT * 2);
            f32x4 bev[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) bev[j] = *(const f32x4*)(Bs + 128 + wid * 32 + j * 16 + fq * 4);
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                f32x4 ae[BT_FE][2];
#pragma unroll
                for (int i = 0; i < BT_FE; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) ae[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < L::KE; ++ks)
#pragma unroll
                    for (int i = 0; i < BT_FE; ++i) {
                        const int q = min((half * BT_FE + i) * 16 + frl, BT_P2 - 1);
                        bf16x8 av;
                        if (ks < 2) {
                            av = *(const bf16x8*)(T2 + q * BT_PITCH + ks * 64 + fq * 16);
                        } else {   // the shortcut's K-source: the window's centre pixel of q
                            const int r = q / BT_TW, c = q - r * BT_TW;
                            av = *(const bf16x8*)(X + xw_off<CIN>((r + 1) * BT_WW + (c + 1), (ks - 2) * 4 + fq));
                        }
#pragma unroll
                        for (int j = 0; j < 2; ++j)
                            ae[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wef[j][ks], av, ae[i][j], 0, 0, 0);
                    }
#pragma unroll
                for (int i = 0; i < BT_FE; ++i) {
                    const int q = (half * BT_FE + i) * 16 + frl;
                    const int r = q / BT_TW, c = q - r * BT_TW;
                    const int h = h0 + r, w = w0 + c;
                    const bool ok = q < BT_P2 && h < H && w < W;
                    const int off = ok ? ((h * W + w) * BT_COUT + wid * 32 + fq * 4) * 2 : 0x7fffff00;
#pragma unroll
                    for (int j = 0; j < 2; ++j) {
                        bf16x4 o;
#pragma unroll
                        for (int k = 0; k < 4; ++k) o[k] = f2bf(fmaxf(ae[i][j][k] + bev[j][k], 0.f));
                        if (BT_EXP != 4) raw_buffer_store_v2i32(__builtin_bit_cast(i32x2, o), yr, off + j * 32, 0, 0);
                        else asm volatile("" :: "v"(o));
                    }
                }
            }
        }
    }
}

int num_cus_bt() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    }
    return n;
}

}  // namespace

hipError_t cbw_bottleneck_s1(const uint16_t* x, uint16_t* y, const uint16_t* wr, const float* br, const uint16_t* wm,
                             const float* bm, const uint16_t* we, const float* be, const void* zero, int N, int H,
                             int W, hipStream_t st) {
    if (N <= 0 || H <= 0 || W <= 0) return hipSuccess;
    const int nrt = (H + BT_TH - 1) / BT_TH, nct = (W + BT_TW - 1) / BT_TW;
    const int64_t nt = (int64_t)N * nrt * nct;
    if (nt >= (1LL << 31) || (int64_t)H * W * BT_COUT * 2 >= 0x7fffff00LL) return hipErrorInvalidValue;
    const int G = (int)std::min<int64_t>(nt, num_cus_bt());
    hipLaunchKernelGGL(bottleneck_s1_kernel, dim3(G), dim3(512), BT_LDS, st, (const bf16*)x, (bf16*)y,
                       (const bf16*)wr, br, (const bf16*)wm, bm, (const bf16*)we, be, zero, N, H, W, nrt, nct);
    return hipGetLastError();
}

hipError_t cbw_bottleneck_s1_first(const uint16_t* x, uint16_t* y, const uint16_t* wr, const float* br,
                                   const uint16_t* wm, const float* bm, const uint16_t* wcat, const float* bcat,
                                   const void* zero, int N, int H, int W, hipStream_t st) {
    if (N <= 0 || H <= 0 || W <= 0) return hipSuccess;
    const int nrt = (H + BT_TH - 1) / BT_TH, nct = (W + BT_TW - 1) / BT_TW;
    const int64_t nt = (int64_t)N * nrt * nct;
    if (nt >= (1LL << 31) || (int64_t)H * W * BT_COUT * 2 >= 0x7fffff00LL) return hipErrorInvalidValue;
    const int G = (int)std::min<int64_t>(nt, num_cus_bt());
    hipLaunchKernelGGL(bottleneck_s1_first_kernel, dim3(G), dim3(512), BtL<64>::LDS, st, (const bf16*)x, (bf16*)y,
                       (const bf16*)wr, br, (const bf16*)wm, bm, (const bf16*)wcat, bcat, zero, N, H, W, nrt, nct);
    return hipGetLastError();
}
