// Implicit-GEMM convolution / GEMM for gfx950 (bf16 MFMA 16x16x32, fp32 accumulate).
//
// One kernel family serves every dense contraction on the CB-Whisper path:
//   * ResNet bottleneck/basic convs (1x1, 3x3, stride 1/2, BN folded into
//     weights + bias) -- HF ResNetConvLayer / ResNetShortCut as called by
//     src/efficient_kws/resnet.py:51-58;
//   * Whisper encoder conv1/conv2 (1x3 over time) and every nn.Linear
//     (projector MLP src/efficient_kws/model.py:87-104, encoder QKV / out / fc1 / fc2).
//
// Layout: activations NHWC bf16 (a Linear is H = 1, W = rows), weights
// [Cout][KH][KW][Cin] bf16 so both MFMA operands are K-contiguous.
// GEMM view: M = N*Ho*Wo output pixels, N = Cout, K = KH*KW*Cin, K-step 64
// (Cin % 64 == 0, Cout % BN == 0 required; the host checks).
//
// Structure (cdna_hip_programming.md §5 minimum 2-phase): A and B tiles are
// gathered straight into LDS with global_load_lds_dwordx4 (per-lane source =
// im2col gather; padding taps read a zero page), double-buffered, XOR swizzle
// on the source chunk so the ds_read_b128 fragment reads are conflict-free;
// 4 waves, each owning a 64x64 output tile (4x4 MFMA tiles); XCD-aware tile
// remap; epilogue staged through LDS so bias/residual/activation and the
// stores run on 16-byte row vectors.
#include "cbw_common.h"
#include "cbw_kernels.h"

thread_local const char* cbw_last_conv_kernel = "";

namespace {

constexpr int BK = 64;             // K elements per stage (128 B per row)
constexpr int EPI_LD = 68;         // fp32 row pitch of the epilogue image (bank-conflict pad)
constexpr int EPI_BYTES = 4 * 64 * EPI_LD * 4;   // 69632: 4 waves x [64][EPI_LD] fp32
template <int BM, int BN>
constexpr int lds_bytes() { return 2 * (BM + BN) * 128 > EPI_BYTES ? 2 * (BM + BN) * 128 : EPI_BYTES; }

CBW_DEV int swz(int r) { return (r >> 1) & 7; }

// epilogue store of output channels col..col+7 of row m (bf16, fp32, or the compensated [hi | hi | lo] split)
CBW_DEV void store_out8(const ConvArgs& a, int flags, int m, int col, const float (&v)[8]) {
    if (flags & CBW_EPI_SPLIT3) {
        bf16x8 hi, lo;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            hi[q] = f2bf(v[q]);
            lo[q] = f2bf(v[q] - bf2f(hi[q]));
        }
        bf16* yp = (bf16*)a.y + (int64_t)m * a.y_ld + col;
        *(bf16x8*)yp = hi;
        *(bf16x8*)(yp + a.Cout) = lo;
        if (a.y32) {
            float* fp = a.y32 + (int64_t)m * a.Cout + col;
            *(f32x4*)fp = f32x4{v[0], v[1], v[2], v[3]};
            *(f32x4*)(fp + 4) = f32x4{v[4], v[5], v[6], v[7]};
        }
    } else if (flags & CBW_EPI_OUT_F32) {
        float* yp = (float*)a.y + (int64_t)m * a.y_ld + col;
        *(f32x4*)yp = f32x4{v[0], v[1], v[2], v[3]};
        *(f32x4*)(yp + 4) = f32x4{v[4], v[5], v[6], v[7]};
    } else {
        bf16x8 o;
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = f2bf(v[q]);
        *(bf16x8*)((bf16*)a.y + (int64_t)m * a.y_ld + col) = o;
    }
}

// residual of output channels col..col+7 of row m from a [hi | lo] tensor (CBW_EPI_RES_SPLIT)
CBW_DEV void res_split8(const ConvArgs& a, int m, int col, float (&rv)[8]) {
    const bf16* rp = (const bf16*)a.res + (int64_t)m * a.res_ld + col;
    const bf16x8 hi = *(const bf16x8*)rp, lo = *(const bf16x8*)(rp + a.Cout);
#pragma unroll
    for (int q = 0; q < 8; ++q) rv[q] = bf2f(hi[q]) + bf2f(lo[q]);
}

// physical channel offset of K-channel c0 (CBW_EPI_SPLIT3 inputs: [hi | lo] read as [hi | hi | lo])
CBW_DEV int fold_c(int c0, int xfold) { return (xfold && c0 >= xfold) ? c0 - xfold : c0; }

template <int BM, int BN, int KH, int KW>
__global__ __launch_bounds__(256, 2) void conv_igemm_kernel(ConvArgs a) {
    static_assert((BM / 64) * (BN / 64) == 4, "4 waves x 64x64 tiles");
    static_assert(KH * KW <= 32, "tap mask");
    constexpr int STAGE = (BM + BN) * 128;
    constexpr int WN = BN / 64;
    constexpr int AR = BM / 32;    // A rows-blocks (8 rows each) per wave per stage
    constexpr int BR = BN / 32;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int nt_n = a.Cout / BN;
    const int nt_m = (a.M + BM - 1) / BM;
    const int bid = xcd_remap(blockIdx.x, nt_m * nt_n);
    const int tm = bid / nt_n, tn = bid % nt_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int Ktot = KH * KW * a.Cin;
    const int csteps = a.Cin / BK;
    const int nsteps_all = KH * KW * csteps;
    const int HoWo = a.Ho * a.Wo;
    const int xld = a.x_ld ? a.x_ld : a.Cin;
    const int S = a.ksplit > 1 ? a.ksplit : 1;
    const int s_lo = (int)blockIdx.y * nsteps_all / S, s_hi = ((int)blockIdx.y + 1) * nsteps_all / S;

    // per-lane A rows: the address of the row's window origin (ih0, iw0) and its in-image tap mask, computed
    // once; a stage then adds one scalar offset (its tap and channel step advance as scalar state)
    const int sub_r = lane >> 3, chunk = lane & 7;
    const bf16* a_px[AR];
    unsigned a_tm[AR];
#pragma unroll
    for (int j = 0; j < AR; ++j) {
        const int r = (wid * AR + j) * 8 + sub_r;
        const int m = m0 + r;
        const bool okm = m < a.M;
        const int mm = okm ? m : 0;
        const int n = mm / HoWo, rem = mm - n * HoWo;
        const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
        const int ih0 = oh * a.sh - a.ph, iw0 = ow * a.sw - a.pw;
        unsigned tm = 0;
#pragma unroll
        for (int kh = 0; kh < KH; ++kh)
#pragma unroll
            for (int kw = 0; kw < KW; ++kw) {
                const int ih = ih0 + kh, iw = iw0 + kw;
                if (okm && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) tm |= 1u << (kh * KW + kw);
            }
        a_tm[j] = tm;
        a_px[j] = (const bf16*)a.x + (int64_t)n * a.H * a.W * xld + ((int64_t)ih0 * a.W + iw0) * xld +
                  ((chunk ^ swz(r)) * 8);
    }
    int nx_cs = s_lo % csteps, nx_tap = s_lo / csteps;   // the stage the next issue_stage reads
    int nx_kh = nx_tap / KW, nx_kw = nx_tap - nx_kh * KW;
    const bf16* wrow[BR];
#pragma unroll
    for (int j = 0; j < BR; ++j) {
        const int r = (wid * BR + j) * 8 + sub_r;
        wrow[j] = (const bf16*)a.w + (int64_t)(n0 + r) * Ktot + ((chunk ^ swz(r)) * 8);
    }

    auto issue_stage = [&](int s, int buf) {   // s must be the nx_* stage; advances it
        const int tap = nx_tap;
        const int off = (nx_kh * a.W + nx_kw) * xld + fold_c(nx_cs * BK, a.xfold);
        if (++nx_cs == csteps) {
            nx_cs = 0;
            ++nx_tap;
            if (++nx_kw == KW) { nx_kw = 0; ++nx_kh; }
        }
        char* A = smem + buf * STAGE;
        char* B = A + BM * 128;
#pragma unroll
        for (int j = 0; j < AR; ++j) {
            const int rb = wid * AR + j;
            const void* src = ((a_tm[j] >> tap) & 1u) ? (const void*)(a_px[j] + off) : a.zero;
            __builtin_amdgcn_global_load_lds(src, (void*)(A + rb * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < BR; ++j) {
            const int rb = wid * BR + j;
            __builtin_amdgcn_global_load_lds((const void*)(wrow[j] + (int64_t)s * BK), (void*)(B + rb * 1024), 16, 0, 0);
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    issue_stage(s_lo, 0);
    // Epilogue operands are prefetched with stage 0 so their HBM latency overlaps the
    // A/B fetch instead of serialising the store loop: each lane owns columns
    // col..col+7 of rows (it*8 + lane/8), it = 0..7, of its wave's 64x64 tile.
    const int ecg = lane & 7, erow = lane >> 3;
    const int ecol = n0 + wn * 64 + ecg * 8;
    const bool res_bf16 = S == 1 && a.res != nullptr && !(a.flags & (CBW_EPI_RES_F32 | CBW_EPI_RES_SPLIT));
    bf16x8 rpre[8];
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int m = m0 + wm * 64 + it * 8 + erow;
        if (res_bf16 && m < a.M)
            rpre[it] = *(const bf16x8*)((const bf16*)a.res + (int64_t)m * a.res_ld + ecol);
        else
            rpre[it] = bf16x8{};
    }
    f32x4 bias0 = {0.f, 0.f, 0.f, 0.f}, bias1 = {0.f, 0.f, 0.f, 0.f};
    if (a.bias) {
        bias0 = *(const f32x4*)(a.bias + ecol);
        bias1 = *(const f32x4*)(a.bias + ecol + 4);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const int fr = lane & 15, fq = lane >> 4;
    for (int s = s_lo; s < s_hi; ++s) {
        const int buf = (s - s_lo) & 1;
        if (s + 1 < s_hi) issue_stage(s + 1, buf ^ 1);
        const char* A = smem + buf * STAGE;
        const char* B = A + BM * 128;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int g = ks * 4 + fq;
            bf16x8 av[4], bv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = wm * 64 + i * 16 + fr;
                av[i] = *(const bf16x8*)(A + r * 128 + ((g ^ swz(r)) * 16));
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int r = wn * 64 + j * 16 + fr;
                bv[j] = *(const bf16x8*)(B + r * 128 + ((g ^ swz(r)) * 16));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // ---- epilogue: wave-private fp32 image [64][EPI_LD] in LDS ----
    float* E = (float*)smem + wid * 64 * EPI_LD;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                E[(i * 16 + fq * 4 + q) * EPI_LD + j * 16 + fr] = acc[i][j][q];
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): own wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();

    const int flags = a.flags;
    // the residuals not prefetched with stage 0 (fp32, or the compensated tier's [hi | lo] pair): the 8 rows' loads
    // all issued here, unconditionally (clamped rows), as raw 16-byte words -- loaded inside the row loop's branches
    // they went out one round trip after another
    const bool res_wide = S == 1 && a.res != nullptr && (a.flags & (CBW_EPI_RES_F32 | CBW_EPI_RES_SPLIT));
    uint4 rw0[8], rw1[8];
    if (res_wide) {
        const bool split = (flags & CBW_EPI_RES_SPLIT) != 0;
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int mc = min(m0 + wm * 64 + it * 8 + erow, a.M - 1);
            if (split) {
                const bf16* rp = (const bf16*)a.res + (int64_t)mc * a.res_ld + ecol;
                rw0[it] = *(const uint4*)rp;
                rw1[it] = *(const uint4*)(rp + a.Cout);
            } else {
                const float* rp = (const float*)a.res + (int64_t)mc * a.res_ld + ecol;
                rw0[it] = *(const uint4*)rp;
                rw1[it] = *(const uint4*)(rp + 4);
            }
        }
    }
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int r = it * 8 + erow, cg = ecg;
        const int m = m0 + wm * 64 + r;
        if (m >= a.M) continue;
        const int col = ecol;
        const f32x4 e0 = *(const f32x4*)(E + r * EPI_LD + cg * 8);
        const f32x4 e1 = *(const f32x4*)(E + r * EPI_LD + cg * 8 + 4);
        if (S > 1) {   // split-K: raw partial sums, the epilogue runs in splitk_epilogue_kernel
            float* pp = a.partial + ((int64_t)blockIdx.y * a.M + m) * a.Cout + col;
            *(f32x4*)pp = e0;
            *(f32x4*)(pp + 4) = e1;
            continue;
        }
        float v[8] = {e0[0], e0[1], e0[2], e0[3], e1[0], e1[1], e1[2], e1[3]};
#pragma unroll
        for (int q = 0; q < 4; ++q) { v[q] += bias0[q]; v[q + 4] += bias1[q]; }
        float rv[8];
        const bool has_res = a.res != nullptr;
        if (has_res) {
            if (flags & CBW_EPI_RES_SPLIT) {   // res_split8's arithmetic on the prefetched pair
                const bf16x8 hi = __builtin_bit_cast(bf16x8, rw0[it]), lo = __builtin_bit_cast(bf16x8, rw1[it]);
#pragma unroll
                for (int q = 0; q < 8; ++q) rv[q] = bf2f(hi[q]) + bf2f(lo[q]);
            } else if (flags & CBW_EPI_RES_F32) {
                const f32x4 r0 = __builtin_bit_cast(f32x4, rw0[it]), r1 = __builtin_bit_cast(f32x4, rw1[it]);
#pragma unroll
                for (int q = 0; q < 4; ++q) { rv[q] = r0[q]; rv[q + 4] = r1[q]; }
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) rv[q] = bf2f(rpre[it][q]);
            }
            if (!(flags & CBW_EPI_RES_AFTER_ACT))
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] += rv[q];
        }
        if (flags & CBW_EPI_RELU) {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
        } else if (flags & CBW_EPI_GELU) {
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = gelu_erf(v[q]);
        }
        if (has_res && (flags & CBW_EPI_RES_AFTER_ACT))
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] += rv[q];
        store_out8(a, flags, m, col, v);
    }
}

// ---------------------------------------------------------------------------
// Persistent variant: grid = 2 blocks per CU, each block walks tiles
// blockIdx.x, +G, +2G, ... (XCD-aware order) as ONE flattened stream of K-stages,
// so the double-buffered glds prefetch runs across tile boundaries: the next
// tile's first stage and its residual/bias are in flight while the current tile
// finishes its MFMAs and epilogue.  This removes the per-tile load->compute->store
// serialisation that makes the short-K 1x1 convs (K = 64..256, wide Cout, residual)
// HBM-latency-bound.  The epilogue image is wave-private and lives beside the two
// stage buffers (8 rows per round, 8.5 KB), so 2 blocks still fit per CU.
template <int BM, int BN, int KH, int KW>
__global__ __launch_bounds__(256, 2) void conv_igemm_persist(ConvArgs a, int ntiles) {
    static_assert((BM / 64) * (BN / 64) == 4, "4 waves x 64x64 tiles");
    static_assert(KH * KW <= 32, "tap mask");
    constexpr int STAGE = (BM + BN) * 128;
    constexpr int WN = BN / 64;
    constexpr int AR = BM / 32;
    constexpr int BR = BN / 32;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    float* E = (float*)(smem + 2 * STAGE) + wid * 8 * EPI_LD;
    const int nt_n = a.Cout / BN;
    const int cin2 = (KH * KW == 1 && a.x2 != nullptr) ? a.Cin2 : 0;
    const int Ktot = KH * KW * a.Cin + cin2;
    const int csteps = a.Cin / BK;
    const int nsteps = KH * KW * csteps + cin2 / BK;
    const int HoWo = a.Ho * a.Wo;
    const int xld = a.x_ld ? a.x_ld : a.Cin;
    const int G = gridDim.x;
    const int my_tiles = (ntiles - (int)blockIdx.x + G - 1) / G;
    const int total = my_tiles * nsteps;
    const int sub_r = lane >> 3, chunk = lane & 7;
    auto tile_of = [&](int ti) { return xcd_remap(ti * G + (int)blockIdx.x, ntiles); };

    // ---- issue cursor: A-row gather state of the tile whose stages are being issued
    int64_t a_base[AR];
    int64_t a_base2[(KH * KW == 1) ? AR : 1];   // second K-source (strided 1x1) row offsets
    int a_ih0[AR], a_iw0[AR];
    bool a_ok[AR];
    const bf16* wrow[BR];
    const bool dual = (KH * KW == 1) && a.x2 != nullptr;
    const int csteps1 = csteps;                                  // stages from x; the rest from x2
    auto setup_issue_tile = [&](int ti) {
        const int tile = tile_of(ti);
        const int m0 = (tile / nt_n) * BM, n0 = (tile % nt_n) * BN;
#pragma unroll
        for (int j = 0; j < AR; ++j) {
            const int r = (wid * AR + j) * 8 + sub_r;
            const int m = m0 + r;
            a_ok[j] = m < a.M;
            const int mm = a_ok[j] ? m : 0;
            const int n = mm / HoWo, rem = mm - n * HoWo;
            const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
            a_ih0[j] = oh * a.sh - a.ph;
            a_iw0[j] = ow * a.sw - a.pw;
            a_base[j] = (int64_t)n * a.H * a.W * xld;
            if constexpr (KH * KW == 1)
                if (dual) a_base2[j] = (((int64_t)n * a.H2 + oh * a.s2) * a.W2 + ow * a.s2) * a.Cin2;
        }
#pragma unroll
        for (int j = 0; j < BR; ++j) {
            const int r = (wid * BR + j) * 8 + sub_r;
            wrow[j] = (const bf16*)a.w + (int64_t)(n0 + r) * Ktot + ((chunk ^ swz(r)) * 8);
        }
    };
    auto issue_stage = [&](int s, int buf) {
        const int tap = s / csteps;
        const int c0 = fold_c((s - tap * csteps) * BK, a.xfold);
        const int kh = tap / KW, kw = tap - kh * KW;
        char* A = smem + buf * STAGE;
        char* B = A + BM * 128;
        const bool second = dual && s >= csteps1;
#pragma unroll
        for (int j = 0; j < AR; ++j) {
            const int rb = wid * AR + j;
            const int r = rb * 8 + sub_r;
            const void* src;
            const int ih = a_ih0[j] + kh, iw = a_iw0[j] + kw;
            bool ok = a_ok[j];
            if constexpr (KH * KW > 1) ok = ok && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
            if (!ok)
                src = a.zero;
            else if constexpr (KH * KW == 1) {
                if (second)
                    src = (const bf16*)a.x2 + a_base2[j] + (s - csteps1) * BK + ((chunk ^ swz(r)) * 8);
                else
                    src = (const bf16*)a.x + a_base[j] + ((int64_t)ih * a.W + iw) * xld + c0 + ((chunk ^ swz(r)) * 8);
            } else
                src = (const bf16*)a.x + a_base[j] + ((int64_t)ih * a.W + iw) * xld + c0 + ((chunk ^ swz(r)) * 8);
            __builtin_amdgcn_global_load_lds(src, (void*)(A + rb * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < BR; ++j) {
            const int rb = wid * BR + j;
            __builtin_amdgcn_global_load_lds((const void*)(wrow[j] + (int64_t)s * BK), (void*)(B + rb * 1024), 16, 0, 0);
        }
    };

    // ---- epilogue operands of the tile being computed
    const int ecg = lane & 7, erow = lane >> 3;
    const bool res_bf16 = a.res != nullptr && !(a.flags & (CBW_EPI_RES_F32 | CBW_EPI_RES_SPLIT));
    bf16x8 rpre[8];
    f32x4 bias0, bias1;
    auto prefetch_epi = [&](int tile) {
        const int m0 = (tile / nt_n) * BM, n0 = (tile % nt_n) * BN;
        const int ecol = n0 + wn * 64 + ecg * 8;
#pragma unroll
        for (int it = 0; it < 8; ++it) {
            const int m = m0 + wm * 64 + it * 8 + erow;
            if (res_bf16 && m < a.M)
                rpre[it] = *(const bf16x8*)((const bf16*)a.res + (int64_t)m * a.res_ld + ecol);
            else
                rpre[it] = bf16x8{};
        }
        bias0 = f32x4{0.f, 0.f, 0.f, 0.f};
        bias1 = f32x4{0.f, 0.f, 0.f, 0.f};
        if (a.bias) {
            bias0 = *(const f32x4*)(a.bias + ecol);
            bias1 = *(const f32x4*)(a.bias + ecol + 4);
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (total == 0) return;
    setup_issue_tile(0);
    issue_stage(0, 0);
    prefetch_epi(tile_of(0));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const int fr = lane & 15, fq = lane >> 4;
    const int flags = a.flags;
    int s_issue = 0, ti_issue = 0;     // stage / tile of the most recently issued stage
    int ti_comp = 0;
    for (int j = 0; j < total; ++j) {
        const int buf = j & 1;
        if (j + 1 < total) {
            if (++s_issue == nsteps) {
                s_issue = 0;
                setup_issue_tile(++ti_issue);
            }
            issue_stage(s_issue, buf ^ 1);
        }
        const char* A = smem + buf * STAGE;
        const char* B = A + BM * 128;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int g = ks * 4 + fq;
            bf16x8 av[4], bv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = wm * 64 + i * 16 + fr;
                av[i] = *(const bf16x8*)(A + r * 128 + ((g ^ swz(r)) * 16));
            }
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int r = wn * 64 + jj * 16 + fr;
                bv[jj] = *(const bf16x8*)(B + r * 128 + ((g ^ swz(r)) * 16));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[jj], acc[i][jj], 0, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if ((j + 1) % nsteps != 0) continue;

        // ---- epilogue of tile ti_comp: 8 rounds of 8 rows through the wave-private image
        const int tile = tile_of(ti_comp);
        const int m0 = (tile / nt_n) * BM, n0 = (tile % nt_n) * BN;
        const int ecol = n0 + wn * 64 + ecg * 8;
#pragma unroll
        for (int r8 = 0; r8 < 8; ++r8) {
            const int i = r8 >> 1;
            if ((fq >> 1) == (r8 & 1)) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        E[((fq & 1) * 4 + q) * EPI_LD + jj * 16 + fr] = acc[i][jj][q];
            }
            const int m = m0 + wm * 64 + r8 * 8 + erow;
            const f32x4 e0 = *(const f32x4*)(E + erow * EPI_LD + ecg * 8);
            const f32x4 e1 = *(const f32x4*)(E + erow * EPI_LD + ecg * 8 + 4);
            if (m < a.M) {
                float v[8] = {e0[0] + bias0[0], e0[1] + bias0[1], e0[2] + bias0[2], e0[3] + bias0[3],
                              e1[0] + bias1[0], e1[1] + bias1[1], e1[2] + bias1[2], e1[3] + bias1[3]};
                float rv[8];
                const bool has_res = a.res != nullptr;
                if (has_res) {
                    if (flags & CBW_EPI_RES_SPLIT) {
                        res_split8(a, m, ecol, rv);
                    } else if (flags & CBW_EPI_RES_F32) {
                        const float* rp = (const float*)a.res + (int64_t)m * a.res_ld + ecol;
                        const f32x4 r0 = *(const f32x4*)rp, r1 = *(const f32x4*)(rp + 4);
#pragma unroll
                        for (int q = 0; q < 4; ++q) { rv[q] = r0[q]; rv[q + 4] = r1[q]; }
                    } else {
#pragma unroll
                        for (int q = 0; q < 8; ++q) rv[q] = bf2f(rpre[r8][q]);
                    }
                    if (!(flags & CBW_EPI_RES_AFTER_ACT))
#pragma unroll
                        for (int q = 0; q < 8; ++q) v[q] += rv[q];
                }
                if (flags & CBW_EPI_RELU) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
                } else if (flags & CBW_EPI_GELU) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) v[q] = gelu_erf(v[q]);
                }
                if (has_res && (flags & CBW_EPI_RES_AFTER_ACT))
#pragma unroll
                    for (int q = 0; q < 8; ++q) v[q] += rv[q];
                store_out8(a, flags, m, ecol, v);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (++ti_comp < my_tiles) prefetch_epi(tile_of(ti_comp));
    }
}

// ---------------------------------------------------------------------------
// 8-wave variant for the MFMA-bound convs (3x3 and deep-K 1x1): BM = 256 output pixels x
// BN = 128/256 channels per block, BK = 32, a 4-deep LDS ring filled by glds with two
// K-steps kept in flight across the (single, raw) barrier of each K-step: the wait before
// the barrier is a counted vmcnt, never 0 inside the loop (cdna_hip_programming.md §5
// "Pipelining across barriers").  64-byte LDS rows, chunk swizzle c ^ ((4 - (r >> 2)) & 3):
// conflict-free for the ds_read_b128 lane groups at K = 32.
// The MFMA runs transposed (C^T = W . X^T): each lane ends with 4 consecutive output
// channels of one pixel, so the epilogue (bias, ReLU, bf16) stores 8 bytes per lane with no
// LDS staging.
constexpr int BIG_BM = 256;
constexpr int BIG_BK = 32;
constexpr int BIG_NS = 4;
CBW_DEV int swz4(int r) { return (4 - (r >> 2)) & 3; }

// Software-pipelined schedule of the 8-wave ring (conv_igemm_big2): per K-step, all LDS fragment
// reads are issued first, the MFMAs of the first half of the wave's fragments run while the second
// half's reads land, and the next stage's glds issue (address math, VALU) sits between the two MFMA
// halves instead of in front of them -- the MFMA pipe no longer idles through the address math and
// the read latency.  The im2col gather keeps one base pointer and a valid-tap bitmask per A row (set
// once per tile), so each issue is a scalar tap offset plus a bit test.
template <int BN, int KH, int KW>
__global__ __launch_bounds__(512, 1) void conv_igemm_big2(ConvArgs a) {
    constexpr int WN = BN / 64;
    constexpr int WM = 8 / WN;
    constexpr int FM = BIG_BM / WM / 16;
    constexpr int FH = FM / 2;
    constexpr int STAGE = (BIG_BM + BN) * 64;
    constexpr int AG = BIG_BM * 64 / 8192;
    constexpr int BG = BN * 64 / 8192;
    constexpr int G = AG + BG;
    static_assert(KH * KW <= 32, "tap mask");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int nt_n = a.Cout / BN;
    const int nt_m = (a.M + BIG_BM - 1) / BIG_BM;
    const int bid = xcd_remap(blockIdx.x, nt_m * nt_n);
    const int tm = bid / nt_n, tn = bid % nt_n;
    const int m0 = tm * BIG_BM, n0 = tn * BN;
    const int Ktot = KH * KW * a.Cin;
    const int nsteps = KH * KW * (a.Cin / BIG_BK);
    const int HoWo = a.Ho * a.Wo;
    const int xld = a.x_ld ? a.x_ld : a.Cin;   // physical channels per pixel ([hi | lo] inputs: 2/3 of Cin)

    const int sub_r = lane >> 2, chunk = lane & 3;
    const bf16* a_px[AG];
    unsigned a_tm[AG];
#pragma unroll
    for (int j = 0; j < AG; ++j) {
        const int r = j * 128 + wid * 16 + sub_r;
        const int m = m0 + r;
        const bool okm = m < a.M;
        const int mm = okm ? m : 0;
        const int n = mm / HoWo, rem = mm - n * HoWo;
        const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
        const int ih0 = oh * a.sh - a.ph, iw0 = ow * a.sw - a.pw;
        unsigned tmask = 0;
#pragma unroll
        for (int kh = 0; kh < KH; ++kh)
#pragma unroll
            for (int kw = 0; kw < KW; ++kw) {
                const int ih = ih0 + kh, iw = iw0 + kw;
                if (okm && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) tmask |= 1u << (kh * KW + kw);
            }
        a_tm[j] = tmask;
        a_px[j] = (const bf16*)a.x + (int64_t)n * a.H * a.W * xld + ((int64_t)ih0 * a.W + iw0) * xld +
                  ((chunk ^ swz4(r)) * 8);
    }
    const bf16* wrow[BG];
#pragma unroll
    for (int j = 0; j < BG; ++j) {
        const int r = j * 128 + wid * 16 + sub_r;
        wrow[j] = (const bf16*)a.w + (int64_t)(n0 + r) * Ktot + ((chunk ^ swz4(r)) * 8);
    }
    // issue cursor (stage, tap, channel offset)
    int is_s = 0, is_tap = 0, is_c = 0, is_kh = 0, is_kw = 0;
    auto issue_next = [&]() {
        char* A = smem + (is_s & (BIG_NS - 1)) * STAGE;
        char* B = A + BIG_BM * 64;
        const int64_t toff = ((int64_t)is_kh * a.W + is_kw) * xld + fold_c(is_c, a.xfold);
#pragma unroll
        for (int j = 0; j < AG; ++j) {
            const void* src = ((a_tm[j] >> is_tap) & 1u) ? (const void*)(a_px[j] + toff) : a.zero;
            __builtin_amdgcn_global_load_lds(src, (void*)(A + (j * 128 + wid * 16) * 64), 16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < BG; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(wrow[j] + (int64_t)is_s * BIG_BK),
                                             (void*)(B + (j * 128 + wid * 16) * 64), 16, 0, 0);
        ++is_s;
        is_c += BIG_BK;
        if (is_c == a.Cin) {
            is_c = 0;
            ++is_tap;
            if (++is_kw == KW) { is_kw = 0; ++is_kh; }
        }
    };

    f32x4 acc[FM][4];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    issue_next();
    if (nsteps > 1) issue_next();
    if (nsteps > 2) issue_next();
    const int fr = lane & 15, fq = lane >> 4;
    for (int s = 0; s < nsteps; ++s) {
        if (s + 2 < nsteps) {
            if constexpr (G == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        } else if (s + 1 < nsteps) {
            if constexpr (G == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        const char* A = smem + (s & (BIG_NS - 1)) * STAGE;
        const char* B = A + BIG_BM * 64;
        bf16x8 av[FM], bv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int r = wn * 64 + j * 16 + fr;
            bv[j] = *(const bf16x8*)(B + r * 64 + ((fq ^ swz4(r)) * 16));
        }
#pragma unroll
        for (int i = 0; i < FH; ++i) {
            const int r = wm * (FM * 16) + i * 16 + fr;
            av[i] = *(const bf16x8*)(A + r * 64 + ((fq ^ swz4(r)) * 16));
        }
        // first half: fragment i's MFMAs, then the read of fragment i + FH (lands under the MFMAs)
#pragma unroll
        for (int i = 0; i < FH; ++i) {
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv[j], av[i], acc[i][j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            const int r = wm * (FM * 16) + (i + FH) * 16 + fr;
            av[i + FH] = *(const bf16x8*)(A + r * 64 + ((fq ^ swz4(r)) * 16));
        }
        __builtin_amdgcn_sched_barrier(0);
        if (s + 3 < nsteps) issue_next();
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = FH; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv[j], av[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        asm volatile("" ::: "memory");
    }

    const bool relu = a.flags & CBW_EPI_RELU;
    const bool split3 = a.flags & CBW_EPI_SPLIT3;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int col = n0 + wn * 64 + j * 16 + fq * 4;
        const f32x4 bb = a.bias ? *(const f32x4*)(a.bias + col) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            const int m = m0 + wm * (FM * 16) + i * 16 + fr;
            if (m >= a.M) continue;
            f32x4 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                v[q] = acc[i][j][q] + bb[q];
                if (relu) v[q] = fmaxf(v[q], 0.f);
            }
            bf16x4 o;
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = f2bf(v[q]);
            bf16* yp = (bf16*)a.y + (int64_t)m * a.y_ld + col;
            *(bf16x4*)yp = o;
            if (split3) {   // compensated tier: [hi | lo] (+ fp32) -- store_out8's split on 4 channels
                bf16x4 lo;
#pragma unroll
                for (int q = 0; q < 4; ++q) lo[q] = f2bf(v[q] - bf2f(o[q]));
                *(bf16x4*)(yp + a.Cout) = lo;
                if (a.y32) *(f32x4*)(a.y32 + (int64_t)m * a.Cout + col) = v;
            }
        }
    }
}

template <int BN, int KH, int KW>
hipError_t launch_big(const ConvArgs& a, hipStream_t st) {
    const int nt = ((a.M + BIG_BM - 1) / BIG_BM) * (a.Cout / BN);
    constexpr int lds = BIG_NS * (BIG_BM + BN) * 64;
    static const std::string nm = kernel_name("conv_igemm_big2", {BN, KH, KW});
    cbw_last_conv_kernel = nm.c_str();
    hipLaunchKernelGGL((conv_igemm_big2<BN, KH, KW>), dim3(nt), dim3(512), lds, st, a);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// 8-phase ping-pong schedule for the MFMA-bound convs (conv_igemm_p8): BM = BN = 256, BK = 64, 8 waves
// as 2 (M halves, "groups") x 4 (N), each wave 128 pixels x 64 channels = 8 x 4 accumulators.  LDS: two
// K-tile buffers of [A 256 rows | B 256 rows] x 128 B (128 KB), rows XOR-swizzled by (r >> 1) & 7.
// A K-tile is computed in four quadrant phases per wave -- (pixels 0-63, ch ni 0), (0-63, 1), (64-127, 1),
// (64-127, 0) of the wave's tile, 16 MFMAs each -- and every phase is "LDS fragment reads + this phase's
// share of the next K-tile's DMA; barrier; MFMAs; barrier".  Group 1 starts one barrier late, so in every
// interval between barriers one group issues MFMAs while the other (the other wave on each SIMD) reads.
// The next K-tile arrives in four half-tiles, one per phase, in the order its phases first read them:
//   A0' = pixel rows {0-63, 128-191} (quadrant 0), B0 = channels 0-127 (quadrants 0, 3), B1 = 128-255
//   (quadrant 1), A1' = rows {64-127, 192-255} (quadrant 2);
// a wave's channel columns are {32 wc .. +31} in B0 and {128 + 32 wc ..} in B1.  Every DMA is retired by
// its own wave (counted vmcnt(4): everything older than its last two phases) at least one barrier before
// any wave reads it, and refills a half-tile at least two intervals after its last reader
// (cdna_hip_programming.md "Pipelining across barriers" / "Read a staged buffer one phase AFTER the wait").
constexpr int P8_BM = 256, P8_BN = 256, P8_BK = 64;
CBW_DEV int p8_off(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
// The same schedule on 512 x 128 tiles (BN = 128: the stage-2 3x3 convs, Cout 128): each group of four waves is
// 2 (pixels) x 2 (channels) waves of the same 128 x 64 wave tile, A half-tiles are 256 rows (4 DMA instructions per
// lane), B half-tiles 64 rows (1): two 80 KB K-tile buffers = the whole 160 KB LDS.  A K-tile moves 80 KB from L2
// for the MFMAs of 64 KB in the 256 x 256 shape, against 128 KB for four 128 x 128 tiles of the 4-wave kernel.
template <int BN> struct P8Shape {
    static constexpr int BM = 65536 / BN;           // 256 / 512
    static constexpr int NA = BM / 128, NB = BN / 128;   // DMA instructions per lane per A / B half-tile
    static constexpr int WCN = BN / 64;             // waves along N in a group (4 / 2)
    static constexpr int BUF = (BM + BN) * 128;
};
// s_waitcnt vmcnt(N) for a compile-time N
template <int N> CBW_DEV void vm_wait() {
    static_assert(N >= 0 && N <= 15, "vm_wait");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int KH, int KW, int BN = 256>
__global__ __launch_bounds__(512, 1) void conv_igemm_p8(ConvArgs a) {
    static_assert(KH * KW <= 32, "tap mask");
    using S = P8Shape<BN>;
    constexpr int BM = S::BM, NA = S::NA, NB = S::NB, WCN = S::WCN;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // wave rows: group (wid >> 2) holds pixel rows BM / 2 * group ..; a wave 128 of them, channels 32 wc .. of each
    // B half-tile (BN = 256: wr = the group, wc = 0..3; BN = 128: two waves along the pixels of each group)
    const int wr = (wid >> 2) * (4 / WCN) + (wid & 3) / WCN, wc = (wid & 3) % WCN;
    const int fr = lane & 15, fq = lane >> 4;
    const int nt_n = a.Cout / BN;
    const int nt_m = (a.M + BM - 1) / BM;
    const int bid = xcd_remap(blockIdx.x, nt_m * nt_n);
    const int tm = bid / nt_n, tn = bid % nt_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int cin2 = a.x2 ? a.Cin2 : 0;             // second K-source (1x1 only): K-tiles past Cin read x2
    const int Ktot = KH * KW * a.Cin + cin2;
    const int csteps = a.Cin / P8_BK;
    const int nk1 = KH * KW * csteps;
    const int nk = nk1 + cin2 / P8_BK;
    const int HoWo = a.Ho * a.Wo;
    const int xld = a.x_ld ? a.x_ld : a.Cin;

    // DMA rows: a wave-instruction fills 8 rows x 128 B (lane -> row + lane / 8, LDS chunk lane % 8, source chunk
    // pre-swizzled).  A half h, instruction g: rows 128 g + 64 h + 8 w ..; B half h, instruction g: 128 h + 64 g + 8 w ..
    const int sub = lane >> 3, pch = lane & 7;
    const bf16* a_px[2][NA];
    const bf16* a2_px[2][NA];
    unsigned a_tm[2][NA];
    const bf16* wrow[2][NB];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int g = 0; g < NA; ++g) {
            const int r = g * 128 + h * 64 + wid * 8 + sub;
            const int m = m0 + r;
            const bool okm = m < a.M;
            const int mm = okm ? m : 0;
            const int n = mm / HoWo, rem = mm - n * HoWo;
            const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
            const int ih0 = oh * a.sh - a.ph, iw0 = ow * a.sw - a.pw;
            a2_px[h][g] = a.x2 ? (const bf16*)a.x2 + (((int64_t)n * a.H2 + oh * a.s2) * a.W2 + ow * a.s2) * cin2 +
                                     ((pch ^ ((r >> 1) & 7)) * 8)
                               : nullptr;
            unsigned tmask = 0;
#pragma unroll
            for (int kh = 0; kh < KH; ++kh)
#pragma unroll
                for (int kw = 0; kw < KW; ++kw) {
                    const int ih = ih0 + kh, iw = iw0 + kw;
                    if (okm && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) tmask |= 1u << (kh * KW + kw);
                }
            a_tm[h][g] = tmask;
            a_px[h][g] = (const bf16*)a.x + (int64_t)n * a.H * a.W * xld + ((int64_t)ih0 * a.W + iw0) * xld +
                         ((pch ^ ((r >> 1) & 7)) * 8);
        }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int g = 0; g < NB; ++g) {
            const int rb = h * (BN / 2) + g * 64 + wid * 8 + sub;
            // LDS B row rb = 32 q + 16 j + rho holds weight row 32 q + 8 (rho >> 2) + 4 j + (rho & 3): the MFMA output
            // rows 4 fq .. + 3 of a wave's two 16-channel tiles j are then channels 8 fq .. + 7 of its 32, so the
            // epilogue stores 16 bytes per lane (8-byte stores left the store tail issue-bound)
            const int rs = (rb & ~31) | (((rb & 15) >> 2) << 3) | (((rb >> 4) & 1) << 2) | (rb & 3);
            wrow[h][g] = (const bf16*)a.w + (int64_t)(n0 + rs) * Ktot + ((pch ^ ((rb >> 1) & 7)) * 8);
        }
    // The A K-tiles walk (tap, channel step) in order, so the next K-tile's tap and input offset are kept as
    // scalar state advanced once per K-tile (no per-issue divisions / 64-bit products: SQ_ACTIVE_INST_SCA was
    // 10-11 % of the wave cycles with them).  nx_*: the K-tile the next A issues read.
    int nx_cs = 0, nx_tap = 0, nx_kh = 0, nx_kw = 0;
    int nx_off = fold_c(0, a.xfold);   // (kh * W + kw) * xld + channel offset: < 2^31 at every shape taken
    auto advance = [&]() {
        if (++nx_cs == csteps) {
            nx_cs = 0;
            ++nx_tap;
            if (++nx_kw == KW) { nx_kw = 0; ++nx_kh; }
        }
        nx_off = (nx_kh * a.W + nx_kw) * xld + fold_c(nx_cs * P8_BK, a.xfold);
    };
    // half-tile `which` (0 A0', 1 B0, 2 B1, 3 A1') of K-tile kt -> buffer kt & 1 (A halves: kt must be nx's)
    auto issue = [&](int kt, int which) {
        char* A = smem + (kt & 1) * S::BUF;
        if (which == 0 || which == 3) {
            const int h = which == 3;
            if (kt >= nk1) {   // second K-source: 1x1, rows past M masked by tap bit 0
                const int c0 = (kt - nk1) * P8_BK;
#pragma unroll
                for (int g = 0; g < NA; ++g) {
                    const void* src = (a_tm[h][g] & 1u) ? (const void*)(a2_px[h][g] + c0) : a.zero;
                    __builtin_amdgcn_global_load_lds(src, (void*)(A + (g * 128 + h * 64 + wid * 8) * 128), 16, 0, 0);
                }
                return;
            }
            const int tap = nx_tap;
            const int toff = nx_off;
#pragma unroll
            for (int g = 0; g < NA; ++g) {
                const void* src = ((a_tm[h][g] >> tap) & 1u) ? (const void*)(a_px[h][g] + toff) : a.zero;
                __builtin_amdgcn_global_load_lds(src, (void*)(A + (g * 128 + h * 64 + wid * 8) * 128), 16, 0, 0);
            }
        } else {
            const int h = which - 1;
            char* B = A + BM * 128;
#pragma unroll
            for (int g = 0; g < NB; ++g)
                __builtin_amdgcn_global_load_lds((const void*)(wrow[h][g] + (int64_t)kt * P8_BK),
                                                 (void*)(B + (h * (BN / 2) + g * 64 + wid * 8) * 128), 16, 0, 0);
        }
    };

    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 av[4][2], bv[2][2];

#pragma unroll
    for (int w = 0; w < 4; ++w) issue(0, w);
    advance();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wid >= 4) __builtin_amdgcn_s_barrier();   // group 1 runs one barrier behind
    for (int kt = 0; kt < nk; ++kt) {
        const char* A = smem + (kt & 1) * S::BUF;
        const char* B = A + BM * 128;
        const bool more = kt + 1 < nk;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int mi = q >> 1, ni = (q == 1 || q == 2) ? 1 : 0;
            // ---- load phase: this phase's share of the next K-tile, then the quadrant's fragments.  The counted
            // wait leaves this phase's and the previous phase's half-tiles in flight (NA + NA, NB + NA, NB + NB,
            // NA + NB instructions after phases 0..3)
            __builtin_amdgcn_sched_barrier(0);
            if (more) {
                issue(kt + 1, q);
                if (q == 3) advance();
                if (q == 0) vm_wait<2 * NA>();
                else if (q == 2) vm_wait<2 * NB>();
                else vm_wait<NA + NB>();
            } else if (q == 0) {
                vm_wait<NA>();
            } else {
                vm_wait<0>();
            }
            if (q == 0 || q == 2) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int ks = 0; ks < 2; ++ks)
                        av[i][ks] = *(const bf16x8*)(A + p8_off(wr * 128 + mi * 64 + i * 16 + fr, ks * 4 + fq));
            }
            if (q != 2) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int ks = 0; ks < 2; ++ks)
                        bv[j][ks] = *(const bf16x8*)(B + p8_off(ni * (BN / 2) + wc * 32 + j * 16 + fr, ks * 4 + fq));
            }
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            // ---- MFMA phase: quadrant (mi, ni), K = 64
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[mi * 4 + i][ni * 2 + j] =
                            __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv[j][ks], av[i][ks], acc[mi * 4 + i][ni * 2 + j], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
        }
    }
    if (wid < 4) __builtin_amdgcn_s_barrier();   // equal barrier counts for both groups

    // epilogue: lane holds channels n0 + 128 ni + 32 wc + 8 fq .. + 7 (acc[.][2 ni] then acc[.][2 ni + 1], 4 each) of
    // pixel m0 + 128 wr + 16 f + fr.  The tile kernels' epilogue arithmetic (bias, then the residual -- bf16, the
    // compensated tier's [hi | lo] pair or fp32 --, then ReLU) and their store_out8 (bf16, [hi | lo] split with the
    // optional fp32 copy, or fp32): the same outputs bit for bit.  A half's 8 residual rows are loaded before any of
    // its stores (clamped rows; loaded inside the row loop they went out one round trip after another).
    const int flags = a.flags;
    const bool relu = flags & CBW_EPI_RELU;
    const bool has_res = a.res != nullptr;
    const bool res_split = flags & CBW_EPI_RES_SPLIT, res_f32 = flags & CBW_EPI_RES_F32;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
        const int col = n0 + ni * (BN / 2) + wc * 32 + fq * 8;
        f32x4 bb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        if (a.bias) {
            bb[0] = *(const f32x4*)(a.bias + col);
            bb[1] = *(const f32x4*)(a.bias + col + 4);
        }
        uint4 rw0[8], rw1[8];
        if (has_res) {
#pragma unroll
            for (int f = 0; f < 8; ++f) {
                const int mc = min(m0 + wr * 128 + f * 16 + fr, a.M - 1);
                if (res_f32) {
                    const float* rp = (const float*)a.res + (int64_t)mc * a.res_ld + col;
                    rw0[f] = *(const uint4*)rp;
                    rw1[f] = *(const uint4*)(rp + 4);
                } else {
                    const bf16* rp = (const bf16*)a.res + (int64_t)mc * a.res_ld + col;
                    rw0[f] = *(const uint4*)rp;
                    if (res_split) rw1[f] = *(const uint4*)(rp + a.Cout);
                }
            }
        }
#pragma unroll
        for (int f = 0; f < 8; ++f) {
            const int m = m0 + wr * 128 + f * 16 + fr;
            if (m >= a.M) continue;
            float v[8];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) v[4 * j + q] = acc[f][ni * 2 + j][q] + bb[j][q];
            if (has_res) {
                float rv[8];
                if (res_split) {
                    const bf16x8 hi = __builtin_bit_cast(bf16x8, rw0[f]), lo = __builtin_bit_cast(bf16x8, rw1[f]);
#pragma unroll
                    for (int q = 0; q < 8; ++q) rv[q] = bf2f(hi[q]) + bf2f(lo[q]);
                } else if (res_f32) {
                    const f32x4 r0 = __builtin_bit_cast(f32x4, rw0[f]), r1 = __builtin_bit_cast(f32x4, rw1[f]);
#pragma unroll
                    for (int q = 0; q < 4; ++q) { rv[q] = r0[q]; rv[q + 4] = r1[q]; }
                } else {
                    const bf16x8 r = __builtin_bit_cast(bf16x8, rw0[f]);
#pragma unroll
                    for (int q = 0; q < 8; ++q) rv[q] = bf2f(r[q]);
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] += rv[q];
            }
            if (relu)
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = fmaxf(v[q], 0.f);
            store_out8(a, flags, m, col, v);
        }
    }
}

template <int KH, int KW, int BN = 256>
hipError_t launch_p8(const ConvArgs& a, hipStream_t st) {
    using S = P8Shape<BN>;
    if (BN != 256) {   // 160 KB of dynamic LDS
        static const hipError_t attr = hipFuncSetAttribute((const void*)conv_igemm_p8<KH, KW, BN>,
                                                           hipFuncAttributeMaxDynamicSharedMemorySize, 2 * S::BUF);
        if (attr != hipSuccess) return attr;
    }
    static const std::string nm = kernel_name("conv_igemm_p8", {KH, KW, BN});
    cbw_last_conv_kernel = nm.c_str();
    const int nt = ((a.M + S::BM - 1) / S::BM) * (a.Cout / BN);
    hipLaunchKernelGGL((conv_igemm_p8<KH, KW, BN>), dim3(nt), dim3(512), 2 * S::BUF, st, a);
    return hipGetLastError();
}

// CBW_CONV_P8 (default 1): the 8-phase kernel for the convs conv_igemm_big2 would run (Cout % 256, Cin % 64).
// tools/layer_bench.py, 625 LEF pairs, big2 -> p8: stage-3 reduce 136 -> 118 us, stage-4 first reduce 231 -> 185,
// stage-3 first 3x3 230 -> 204, other 3x3s within +-1.5 %; bench.py 4.59 -> 4.72 utt/s (two rounds each)
int p8_x2() {   // CBW_P8_X2: 0 never, 1 the x2 convs ring / persist would run, 2 also those on the streaming kernel
    const char* e = getenv("CBW_P8_X2");
    return e ? atoi(e) : 1;
}

bool p8_tier_enabled() {
    const char* e = getenv("CBW_P8_TIER");
    return !(e && atoi(e) == 0);
}

int p8_n128() {
    const char* e = getenv("CBW_P8_N128");
    return e ? atoi(e) : 1;
}

int p8_mode() {
    const char* e = getenv("CBW_CONV_P8");
    return e ? atoi(e) : 1;
}

int num_cus() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    }
    return n;
}

template <int BM, int BN, int KH, int KW>
hipError_t launch_persist(const ConvArgs& a, hipStream_t st) {
    const int ntiles = ((a.M + BM - 1) / BM) * (a.Cout / BN);
    int G = 2 * num_cus();
    if (ntiles < G) G = ntiles;
    constexpr int lds = 2 * (BM + BN) * 128 + 4 * 8 * EPI_LD * 4;
    static const std::string nm = kernel_name("conv_igemm_persist", {BM, BN, KH, KW});
    cbw_last_conv_kernel = nm.c_str();
    hipLaunchKernelGGL((conv_igemm_persist<BM, BN, KH, KW>), dim3(G), dim3(256), lds, st, a, ntiles);
    return hipGetLastError();
}

template <int BM, int BN, int KH, int KW>
hipError_t launch_t(const ConvArgs& a, hipStream_t st) {
    const int nt = ((a.M + BM - 1) / BM) * (a.Cout / BN);
    constexpr int lds = lds_bytes<BM, BN>();
    static const std::string nm = kernel_name("conv_igemm_kernel", {BM, BN, KH, KW});
    cbw_last_conv_kernel = nm.c_str();
    hipLaunchKernelGGL((conv_igemm_kernel<BM, BN, KH, KW>), dim3(nt), dim3(256), lds, st, a);
    return hipGetLastError();
}

// The persistent ring kernel (conv_ring.hip) wins where HBM and latency bound the conv: 1x1 convs
// with K <= 768 and no residual (tools/chunk_trace.py, chunk of 500 LEF pairs: stage-2 first-block
// reduce 366 -> 316 us, fused expand+shortcut 424 -> 368 us).  Identity-residual expands stay on
// conv_igemm_persist (2 blocks/CU hide the residual's HBM latency: ring 275 -> 315 us); the
// MFMA-bound ones (3x3, K >= 1024) keep the 256x256 tiles of conv_igemm_big (half the L2 -> LDS
// bytes per FLOP of the ring's 256x128 tile).
bool ring_wanted(const ConvArgs& a) {
    if (!cbw_conv_ring_supported(a)) return false;
    const int ktot = a.KH * a.KW * a.Cin + (a.x2 ? a.Cin2 : 0);
    return a.KH * a.KW == 1 && a.res == nullptr && ktot <= 768;
}

template <int KH, int KW>
hipError_t launch_k(const ConvArgs& a, hipStream_t st) {
    // the tile kernels advance A through a 32-bit scalar offset (tap row/col + channel step): it must fit
    const int64_t xld = a.x_ld ? a.x_ld : a.Cin;
    if (((int64_t)(KH - 1) * a.W + (KW - 1)) * xld + a.Cin + (a.x2 ? a.Cin2 : 0) > INT32_MAX) return hipErrorInvalidValue;
    const bool tile_only = a.xfold || (a.x_ld && a.x_ld != a.Cin) || (a.flags & (CBW_EPI_SPLIT3 | CBW_EPI_RES_SPLIT));
    const bool p8_fit = p8_mode() == 1 && a.res == nullptr && a.Cout % P8_BN == 0 && a.Cin % P8_BK == 0 &&
                        a.xfold % P8_BK == 0 && KH * KW * a.Cin + (a.x2 ? a.Cin2 : 0) >= 512 &&
                        (a.x2 == nullptr || (KH * KW == 1 && a.Cin2 % P8_BK == 0 && !a.xfold && !a.x_ld)) &&
                        !(a.flags & (CBW_EPI_OUT_F32 | CBW_EPI_GELU | CBW_EPI_RES_SPLIT)) &&
                        ((a.M + P8_BM - 1) / P8_BM) * (a.Cout / P8_BN) >= num_cus();
    // folded expand + shortcut (x2): ring / persist -> p8 (CBW_P8_X2 >= 1), streaming -> p8 (CBW_P8_X2 = 2)
    const int px2 = p8_x2();
    if (p8_fit && a.x2 && px2 >= 2) return launch_p8<KH, KW>(a, st);
    if (!tile_only && KH * KW == 1 && cbw_conv_stream_wanted(a)) return cbw_conv_stream(a, st);
    if (p8_fit && a.x2 && px2 >= 1) return launch_p8<KH, KW>(a, st);
    // the compensated tier's convs (CBW_EPI_SPLIT3) at 256 x 256 tiles ("run the tier's stages 3-4
    // at larger tiles"): its expand convs with the [hi | lo] / fp32 residual and its fp32-output shortcuts on p8's
    // residual epilogue, and deep-K convs (K >= 4096: stage 4 at ~400 band pairs, 226 tiles) from half a round of
    // tiles -- one p8 tile's long K loop outruns four 128 x 128 tiles there.  CBW_P8_TIER=0: the tile kernels.
    if (p8_tier_enabled() && (a.flags & (CBW_EPI_SPLIT3 | CBW_EPI_OUT_F32)) && a.xfold && a.x2 == nullptr &&
        p8_mode() == 1 && a.Cout % P8_BN == 0 && a.Cin % P8_BK == 0 && a.xfold % P8_BK == 0 &&
        !(a.flags & (CBW_EPI_GELU | CBW_EPI_RES_AFTER_ACT))) {
        const int ktot = KH * KW * a.Cin;
        const int tiles = ((a.M + P8_BM - 1) / P8_BM) * (a.Cout / P8_BN);
        if (ktot >= 512 && (tiles >= num_cus() || (ktot >= 4096 && 2 * tiles >= num_cus())))
            return launch_p8<KH, KW>(a, st);
    }
    if (!tile_only && ring_wanted(a)) return cbw_conv_ring(a, st);
    // MFMA-bound shapes (K >= 256, no residual, bf16 out, no second K-source) -> 8-wave ring kernel
    // (conv_igemm_big2 also takes the compensated tier's [hi | lo] inputs and split outputs -- x_ld, xfold,
    // CBW_EPI_SPLIT3 -- so its 3x3 and deep-K 1x1 convs run on the same kernel as the bf16 pass)
    const bool big_ok = a.res == nullptr && a.x2 == nullptr &&
                        !(a.flags & (CBW_EPI_OUT_F32 | CBW_EPI_GELU | CBW_EPI_RES_SPLIT)) &&
                        a.Cin % BIG_BK == 0 && a.xfold % BIG_BK == 0 && KH * KW * a.Cin >= 256;
    const int big_tiles = ((a.M + BIG_BM - 1) / BIG_BM) * (a.Cout / 256);
    // (stage 4's 282 tiles fill 1.1 rounds, but the 4-wave kernel there loses more in the two-stream bench
    // than the tail costs: 5.57 vs 5.69 utt/s)
    if (big_ok && big_tiles >= num_cus()) {
        // (a 128-wide tile for the few-tile stage-4 convs -- 282 tiles = 1.1 rounds at LEF -- fills the
        // rounds better but loses more per tile: 5.18 -> 5.05 utt/s in bench.py; not taken)
        // 256-wide tiles only: at Cout = 128 (the stage-2 3x3s) the 4-wave 128x128 kernel below is faster
        // (tools/layer_bench.py: 184 vs 202 us stride 1, 229 vs 237 us stride 2; bench.py +0.6 %)
        if (a.Cout % 256 == 0 && p8_mode() == 1 && a.Cin % P8_BK == 0 && a.xfold % P8_BK == 0)
            return launch_p8<KH, KW>(a, st);
        if (a.Cout % 256 == 0) return launch_big<256, KH, KW>(a, st);
    }
    // Cout 128 (the stage-2 3x3s): the 8-phase schedule on 512 x 128 tiles (CBW_P8_N128=0: the 4-wave kernel below)
    if (big_ok && p8_n128() && p8_mode() == 1 && a.Cout % 256 == 128 && a.Cin % P8_BK == 0 && a.xfold % P8_BK == 0 &&
        KH * KW * a.Cin >= 512 && ((a.M + 511) / 512) * (a.Cout / 128) >= num_cus())
        return launch_p8<KH, KW, 128>(a, st);
    // tile shape: keep BN <= Cout; prefer the 128x128 tile when it divides Cout
    if (a.Cout % 128 == 0) {
        // persistent cross-tile pipelining pays where the per-tile prologue/epilogue is not
        // amortised: a single K-stage, or a residual read in the epilogue (tools/layer_bench.py:
        // S1 expand 493 -> 404 us, S2 expand 298 -> 267 us); deep-K tiles keep the 1-tile kernel.
        const bool short_k = a.KH * a.KW * (a.Cin / BK) == 1;
        if (a.x2 != nullptr || short_k || a.res != nullptr)
            return launch_persist<128, 128, KH, KW>(a, st);
        return launch_t<128, 128, KH, KW>(a, st);
    }
    if (a.x2 != nullptr) return hipErrorInvalidValue;   // dual-source needs Cout % 128 == 0
    return launch_t<256, 64, KH, KW>(a, st);
}

}  // namespace

namespace {
// y = act(sum_z partial[z] + bias (+ res)) over [M][Cout], z summed in order (deterministic); 4 columns per thread
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(ConvArgs a, int S) {
    const int64_t n4 = (int64_t)a.M * a.Cout / 4;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n4; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e * 4;
        const int m = (int)(i / a.Cout), col = (int)(i - (int64_t)m * a.Cout);
        f32x4 v = *(const f32x4*)(a.partial + i);
        for (int z = 1; z < S; ++z) v += *(const f32x4*)(a.partial + (int64_t)z * a.M * a.Cout + i);
        if (a.bias) v += *(const f32x4*)(a.bias + col);
        float rv[4] = {0.f, 0.f, 0.f, 0.f};
        const bool has_res = a.res != nullptr;
        if (has_res) {
            if (a.flags & CBW_EPI_RES_F32) {
                const f32x4 r = *(const f32x4*)((const float*)a.res + (int64_t)m * a.res_ld + col);
#pragma unroll
                for (int q = 0; q < 4; ++q) rv[q] = r[q];
            } else {
                const bf16x4 r = *(const bf16x4*)((const bf16*)a.res + (int64_t)m * a.res_ld + col);
#pragma unroll
                for (int q = 0; q < 4; ++q) rv[q] = bf2f(r[q]);
            }
            if (!(a.flags & CBW_EPI_RES_AFTER_ACT))
#pragma unroll
                for (int q = 0; q < 4; ++q) v[q] += rv[q];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (a.flags & CBW_EPI_RELU) v[q] = fmaxf(v[q], 0.f);
            else if (a.flags & CBW_EPI_GELU) v[q] = gelu_erf(v[q]);
            if (has_res && (a.flags & CBW_EPI_RES_AFTER_ACT)) v[q] += rv[q];
        }
        if (a.flags & CBW_EPI_OUT_F32) {
            *(f32x4*)((float*)a.y + (int64_t)m * a.y_ld + col) = v;
        } else {
            bf16x4 o;
#pragma unroll
            for (int q = 0; q < 4; ++q) o[q] = f2bf(v[q]);
            *(bf16x4*)((bf16*)a.y + (int64_t)m * a.y_ld + col) = o;
        }
    }
}
}  // namespace

int cbw_conv_splitk_factor(const ConvArgs& a) {
    if (a.KH != 1 || a.KW != 1 || a.x2 != nullptr || a.Cout % 128 || a.Cin % BK) return 1;
    const int tiles = ((a.M + 127) / 128) * (a.Cout / 128);
    const int slots = 2 * num_cus();               // conv_igemm_kernel: 2 blocks per CU
    const int nsteps = a.Cin / BK;
    int S = 1;
    while (S < 8 && tiles * (S * 2) <= slots && nsteps / (S * 2) >= 4) S *= 2;
    return S;
}

hipError_t cbw_conv_igemm_splitk(const ConvArgs& a0, int ksplit, float* partial, hipStream_t st) {
    if (ksplit <= 1 || partial == nullptr) return cbw_conv_igemm(a0, st);
    if (a0.KH != 1 || a0.KW != 1 || a0.x2 != nullptr || a0.Cout % 128 || a0.Cin % BK || a0.Cout % 4 ||
        a0.y_ld % 4 || (a0.res && a0.res_ld % 4) || ksplit > a0.Cin / BK)
        return hipErrorInvalidValue;
    ConvArgs a = a0;
    a.ksplit = ksplit;
    a.partial = partial;
    const int nt = ((a.M + 127) / 128) * (a.Cout / 128);
    constexpr int lds = lds_bytes<128, 128>();
    cbw_last_conv_kernel = "conv_igemm_kernel<128, 128, 1, 1> + splitk_epilogue_kernel";
    hipLaunchKernelGGL((conv_igemm_kernel<128, 128, 1, 1>), dim3(nt, ksplit), dim3(256), lds, st, a);
    const int64_t n4 = (int64_t)a.M * a.Cout / 4;
    const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 4 * num_cus());
    hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(grid), dim3(256), 0, st, a, ksplit);
    return hipGetLastError();
}

hipError_t cbw_conv_igemm(const ConvArgs& a, hipStream_t st) {
    if (a.x2 != nullptr && (a.KH != 1 || a.KW != 1 || a.Cin2 % BK)) return hipErrorInvalidValue;
    if (a.KH == 1 && a.KW == 1) return launch_k<1, 1>(a, st);
    if (a.KH == 3 && a.KW == 3) return launch_k<3, 3>(a, st);
    if (a.KH == 1 && a.KW == 3) return launch_k<1, 3>(a, st);
    return hipErrorInvalidValue;
}
