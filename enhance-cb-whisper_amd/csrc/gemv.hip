// Skinny GEMM ("GEMV") for the Whisper decoder step on gfx950: y[m][n] = act(sum_k x[m][k] W[n][k] + b[n]
// (+ res[m][n])) for M <= 16 rows (the beams of one decode step), every decoder Linear (self q/k/v + out,
// cross q + out, fc1, fc2) and the vocabulary projection (HF WhisperDecoderLayer / proj_out as run by
// PBAWhisper.generate's beam search, src/model/pba_whisper.py:283-338 via HF 4.37 _beam_search).
//
// A decode step reads every decoder weight once (large-v3: 1.6 GB) for 5 rows, so it is HBM- and
// latency-bound; the 128-row implicit-GEMM tiles the step used before put 10-40 workgroups on a
// 1280-wide Linear and reached 0.15 TB/s.  Here:
//   * workgroup = 16 output columns x the whole K, split over its W waves (W = 1..16, so that a wave
//     owns <= 10 k-steps of 32): every weight byte of the workgroup's 16 rows is requested in one burst,
//     16 bytes per lane, before the first MFMA;
//   * each wave runs C^T = W . x^T on mfma_f32_16x16x32_bf16 over its K-slice: the weight fragment
//     (16 columns x 32 k) is the A operand, the rows (zero-padded to 16) the B operand;
//   * the W partial accumulators meet in LDS and wave 0 sums them in wave order (deterministic), then
//     applies bias, residual, activation and the output type.  One launch per Linear, no global
//     partials, no atomics.
#include "cbw_common.h"
#include "cbw_kernels.h"

namespace {

constexpr int GV_BATCH = 10;   // k-steps (of 32) in flight per wave

constexpr int GV_LN_MAXK = 1280;   // LayerNorm prologue: a row is <= 5 f32x4 per lane (Whisper d_model <= 1280)
constexpr int GV_LN_LDS = 48 * 1024;   // + the 16 KB reduction buffer: within the 64 KB default

// LN: the LayerNorm-prologue instance (K <= 1280 -> at most 8 waves, so a wider register budget)
template <bool LN>
__global__ __launch_bounds__(LN ? 512 : 1024) void gemv_kernel(GemvArgs a) {
    __shared__ f32x4 red[16][64];
    extern __shared__ __attribute__((aligned(16))) char gv_dyn[];   // LN prologue: bf16 [M][K + 8]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int W = blockDim.x >> 6;
    const int fr = lane & 15, fq = lane >> 4;
    const int KS = a.K / 32;
    const int k_lo = w * KS / W, k_hi = (w + 1) * KS / W;
    const int c0 = blockIdx.x * 16;
    const int n_ld = min(c0 + fr, a.N - 1);
    const bf16* wr = a.w + (int64_t)n_ld * a.K + fq * 8;
    const bool row_ok = fr < a.M;
    constexpr bool ln = LN;
    const int pitch = a.K + 8;
    const bf16* xr = ln ? (const bf16*)gv_dyn + (row_ok ? fr : 0) * pitch + fq * 8
                        : a.x + (int64_t)(row_ok ? fr : 0) * a.ldx + fq * 8;

    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    bf16x8 wv[GV_BATCH], xv[GV_BATCH];
    int k0 = k_lo;
#pragma unroll
    for (int j = 0; j < GV_BATCH; ++j)
        if (k0 + j < k_hi) wv[j] = __builtin_nontemporal_load((const bf16x8*)(wr + (k0 + j) * 32));   // wave-uniform
    if (ln) {
        // LayerNorm of the M rows into LDS while the first weight burst is in flight: wave w takes rows
        // w, w + W, ..., with layernorm_kernel's arithmetic (same per-lane order, same wave reduction)
        bf16* xs = (bf16*)gv_dyn;
        for (int r = w; r < a.M; r += W) {
            const float* xrow = a.xf + (int64_t)r * a.ldx;
            f32x4 v[GV_LN_MAXK / 256], gg[GV_LN_MAXK / 256], bb[GV_LN_MAXK / 256];
#pragma unroll
            for (int c = 0; c < GV_LN_MAXK / 256; ++c) {   // row, gamma and beta in one round trip
                const int i = lane * 4 + c * 256;
                if (i < a.K) {
                    v[c] = *(const f32x4*)(xrow + i);
                    gg[c] = *(const f32x4*)(a.ln_g + i);
                    bb[c] = *(const f32x4*)(a.ln_b + i);
                }
            }
            float sm = 0.f;
#pragma unroll
            for (int c = 0; c < GV_LN_MAXK / 256; ++c)
                if (lane * 4 + c * 256 < a.K) sm += v[c][0] + v[c][1] + v[c][2] + v[c][3];
            const float mean = wave_sum(sm) / a.K;
            float ss = 0.f;
#pragma unroll
            for (int c = 0; c < GV_LN_MAXK / 256; ++c)
                if (lane * 4 + c * 256 < a.K)
#pragma unroll
                    for (int q = 0; q < 4; ++q) ss += (v[c][q] - mean) * (v[c][q] - mean);
            const float rstd = rsqrtf(wave_sum(ss) / a.K + a.ln_eps);
#pragma unroll
            for (int c = 0; c < GV_LN_MAXK / 256; ++c) {
                const int i = lane * 4 + c * 256;
                if (i < a.K) {
                    bf16x4 ob;
#pragma unroll
                    for (int q = 0; q < 4; ++q) ob[q] = f2bf((v[c][q] - mean) * rstd * gg[c][q] + bb[c][q]);
                    *(bf16x4*)(xs + r * pitch + i) = ob;
                }
            }
        }
        __syncthreads();
    }
    for (;;) {
#pragma unroll
        for (int j = 0; j < GV_BATCH; ++j)
            if (k0 + j < k_hi) xv[j] = row_ok ? *(const bf16x8*)(xr + (k0 + j) * 32) : bf16x8{};
#pragma unroll
        for (int j = 0; j < GV_BATCH; ++j)
            if (k0 + j < k_hi) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wv[j], xv[j], acc, 0, 0, 0);
        k0 += GV_BATCH;
        if (k0 >= k_hi) break;
#pragma unroll
        for (int j = 0; j < GV_BATCH; ++j)
            if (k0 + j < k_hi) wv[j] = __builtin_nontemporal_load((const bf16x8*)(wr + (k0 + j) * 32));
    }
    if (W > 1) {
        red[w][lane] = acc;
        __syncthreads();
        if (w != 0) return;
        for (int ww = 1; ww < W; ++ww) acc += red[ww][lane];
    }
    // lane holds C^T[n = c0 + 4 fq + q][m = fr]
    const int m = fr, n = c0 + fq * 4;
    if (!row_ok || n >= a.N) return;
    f32x4 v = acc;
    if (a.bias) v += *(const f32x4*)(a.bias + n);
    float rv[4] = {0.f, 0.f, 0.f, 0.f};
    const bool has_res = a.res != nullptr;
    if (has_res) {
        if (a.flags & CBW_EPI_RES_F32) {
            const f32x4 r = *(const f32x4*)((const float*)a.res + (int64_t)m * a.res_ld + n);
#pragma unroll
            for (int q = 0; q < 4; ++q) rv[q] = r[q];
        } else {
            const bf16x4 r = *(const bf16x4*)((const bf16*)a.res + (int64_t)m * a.res_ld + n);
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
        *(f32x4*)((float*)a.y + (int64_t)m * a.ldy + n) = v;
    } else {
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] = f2bf(v[q]);
        *(bf16x4*)((bf16*)a.y + (int64_t)m * a.ldy + n) = o;
        if (a.kv_k && n >= a.kv_D) {   // 4 columns never straddle the q/k/v boundaries (kv_D % 4 == 0)
            const int64_t po = a.kv_pos ? (int64_t)a.kv_pos[a.kv_pos_rows ? m : 0] * a.kv_D : 0;
            bf16* dst = (n < 2 * a.kv_D ? a.kv_k + (n - a.kv_D) : a.kv_v + (n - 2 * a.kv_D)) + po;
            *(bf16x4*)(dst + (int64_t)m * a.kv_ld) = o;
        }
    }
}

// VALU variant for the beam rows of a decode step (M <= 16, K % 256 == 0): 2 * WV output columns per workgroup (one
// per wave for the K 5120 fc2), each column's K split over 32 (64) lanes in interleaved 16-byte chunks (a half-wave
// reads 512 contiguous bytes of the weight row per load), every load of the lane's slice issued at once; the M rows
// staged in LDS (LayerNorm prologue or a DMA copy), dot products on v_dot2_f32_bf16, the partial sums reduced by lane
// exchanges in a fixed order (deterministic).  Versus the MFMA kernel above (16 columns per workgroup, 16 - M of its
// 16 B-operand rows padding): 2x the workgroups at the decode step's N (160 at D 1280 instead of 80), so twice the
// CUs stream the weights; the step is latency-bound on the chain of its ~300 launches.
constexpr int GD_MAXM = 8;   // K <= 5120
// 9..16 rows: the 16-row instantiation, its rows staged in up to 158 KB of LDS (gfx950: 160 KB per workgroup)
constexpr int GD_LDS16 = 158 * 1024;
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

template <int N>
CBW_DEV void wait_vm() {   // s_waitcnt vmcnt(N) for the counts the kernel below uses
    static_assert(N == 3 || N == 4 || N == 5 || N == 6 || N == 8 || N == 10 || N == 12 || N == 16 || N == 20 || N == 24 ||
                      N == 32 || N == 40, "count");
    if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if constexpr (N == 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if constexpr (N == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
}

// CPW = output columns per wave: 2 (a column's K over 32 lanes) or 1 (over all 64 lanes: half the weight bytes per
// workgroup, twice the workgroups -- the K 5120 fc2, whose 160 workgroups each staged 51 KB of rows and streamed 80 KB)
// KS = K stages of the DMA'd rows (no LayerNorm): the rows are staged KS times, K / KS columns at a time, so the 16-row
// K 5120 fc2 needs 80 instead of 154 KB of LDS (two workgroups per CU: its 320 workgroups in one round instead of
// two); the sums run over j in the same order, so the results are those of KS = 1 (15-row step 3.44 -> 3.13 ms, r03aj)
// WV = computing waves per workgroup (4, or 8 for the 9..16-row instantiation: each wave's LayerNorm prologue then
// normalises 2 rows instead of 4, and every column is computed by the same lanes in the same order as with 4; 15-row
// step 3.13 -> 2.89 ms, r03al)
template <bool LN, int NJ, int CPW = 2, int MAXM = GD_MAXM, int KS = 1, int WV = 4>
__global__ __launch_bounds__(WV * 64) void gemv_dot_kernel(GemvArgs a) {   // NJ = K / 256; M <= MAXM
    extern __shared__ __attribute__((aligned(16))) char gv_dyn[];   // bf16 [M][K + 8]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int LANES = 64 / CPW, STEP = LANES * 8;   // lanes per column, elements per load step
    constexpr int K = NJ * 256, NL = K / STEP;          // loads per lane
    const int half = CPW == 2 ? lane >> 5 : 0, hl = lane & (LANES - 1);
    static_assert(KS == 1 || (!LN && NL % KS == 0), "K stages: DMA'd rows");
    constexpr int KP = K / KS, NLS = NL / KS;           // columns of K per stage, loads per lane per stage
    const int M = a.M, pitch = LN ? K + 8 : KP;   // the LayerNorm prologue writes padded rows, the DMA packed ones
    const int col = blockIdx.x * (WV * CPW) + w * CPW + half;
    const bf16* wr = a.w + (int64_t)min(col, a.N - 1) * K + hl * 8;
    // the epilogue's operands (bias, residual) do not depend on the sums: requested before anything else, as raw
    // words (no conversion at a branch join, which would wait for the load there), so the epilogue does not start
    // with a dependent round trip
    const int m_e = min(hl, M - 1);
    const bool has_res = a.res != nullptr, res32 = (a.flags & CBW_EPI_RES_F32) != 0;
    const int n_e = min(col, a.N - 1);
    const float bias_raw = *(a.bias ? a.bias + n_e : (const float*)a.w);
    unsigned res_raw = 0;
    if (has_res) {
        const char* rp = (const char*)a.res + ((int64_t)m_e * a.res_ld + n_e) * (res32 ? 4 : 2);
        res_raw = res32 ? *(const unsigned*)rp : (unsigned)*(const unsigned short*)rp;
    }
    // the activations are requested next (L2 round trip), then every weight load of the lane's slice: the
    // counted waits of the activation staging then do not wait behind the weight stream
    bf16x8 wv[NL];
    bf16* xs = (bf16*)gv_dyn;
    if constexpr (LN) {   // LayerNorm of the M rows (layernorm_kernel's arithmetic): wave w takes rows w, w + WV, ...
        constexpr int NC = K / 256;
        static_assert(K <= GV_LN_MAXK, "LayerNorm prologue width");
        constexpr int HS = MAXM / WV;   // row slots per wave: rows w, w + WV, ...
        static_assert(HS >= 1, "row slots");
        f32x4 v[HS][NC], gg[NC], bb[NC];
#pragma unroll
        for (int h = 0; h < HS; ++h) {
            const int r = min(w + WV * h, M - 1);
            const float* xrow = a.xf + (int64_t)r * a.ldx;
#pragma unroll
            for (int c = 0; c < NC; ++c) v[h][c] = *(const f32x4*)(xrow + lane * 4 + c * 256);
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            gg[c] = *(const f32x4*)(a.ln_g + lane * 4 + c * 256);
            bb[c] = *(const f32x4*)(a.ln_b + lane * 4 + c * 256);
        }
#pragma unroll
        for (int j = 0; j < NL; ++j) wv[j] = __builtin_nontemporal_load((const bf16x8*)(wr + j * STEP));
        // both row slots normalised unconditionally (a slot past M repeats row M - 1, its result is not stored): with
        // a conditional second row the compiler sank that row's loads (and gamma / beta) behind the first row's
        // reductions -- three round trips instead of one
#pragma unroll
        for (int h = 0; h < HS; ++h) {
            const int r = w + WV * h;
            float sm = 0.f;
#pragma unroll
            for (int c = 0; c < NC; ++c) sm += v[h][c][0] + v[h][c][1] + v[h][c][2] + v[h][c][3];
            const float mean = wave_sum_x(sm) / K;
            float ss = 0.f;
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
                for (int q = 0; q < 4; ++q) ss += (v[h][c][q] - mean) * (v[h][c][q] - mean);
            const float rstd = rsqrtf(wave_sum_x(ss) / K + a.ln_eps);
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                bf16x4 ob;
#pragma unroll
                for (int q = 0; q < 4; ++q) ob[q] = f2bf((v[h][c][q] - mean) * rstd * gg[c][q] + bb[c][q]);
                if (r < M) *(bf16x4*)(xs + r * pitch + lane * 4 + c * 256) = ob;
            }
        }
    } else {   // the M rows DMA'd straight into LDS (global_load_lds: no registers), every piece in flight at once,
        // then the weight stream; one counted wait for the DMAs leaves the weight loads in flight.  (Staged through
        // registers, the compiler sank each row load next to its LDS store and waited for it before issuing the
        // next: the rows arrived one round trip at a time.)
        const int total = M * KP * 2;                // bytes, rows packed [M][KP] (pitch KP): the first K stage
        const int pieces = (total + 1023) >> 10;     // 1 KB per wave instruction; LDS holds whole pieces
        const int e = lane * 8;                      // this lane's first element within a piece
        for (int pc = w; pc < pieces; pc += WV) {
            const int el = min(pc * 512 + e, M * KP - 8), r = el / KP, c = el - r * KP;
            __builtin_amdgcn_global_load_lds((const void*)(a.x + (int64_t)r * a.ldx + c), (void*)(gv_dyn + pc * 1024),
                                             16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < NL; ++j) wv[j] = __builtin_nontemporal_load((const bf16x8*)(wr + j * STEP));
        // the DMAs were issued before the NL weight loads: vmcnt(NL) retires them (in-order completion)
        wait_vm<NL>();
    }
    __syncthreads();
    float acc[MAXM];
#pragma unroll
    for (int r = 0; r < MAXM; ++r) acc[r] = 0.f;
#pragma unroll
    for (int j = 0; j < NL; ++j) {
        if constexpr (KS > 1) {
            if (j > 0 && j % NLS == 0) {   // the next K stage's rows into the same LDS, once every wave has read these
                __syncthreads();
                const int pieces = (M * KP * 2 + 1023) >> 10, e = lane * 8, k0 = (j / NLS) * KP;
                for (int pc = w; pc < pieces; pc += WV) {
                    const int el = min(pc * 512 + e, M * KP - 8), r = el / KP, c = el - r * KP;
                    __builtin_amdgcn_global_load_lds((const void*)(a.x + (int64_t)r * a.ldx + k0 + c),
                                                     (void*)(gv_dyn + pc * 1024), 16, 0, 0);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
            }
        }
        const bf16x8 wj = wv[j];
#pragma unroll
        for (int r = 0; r < MAXM; ++r) {
            if (r >= M) continue;
            const bf16x8 xv = *(const bf16x8*)(xs + r * pitch + (j % NLS) * STEP + hl * 8);
#pragma unroll
            for (int p = 0; p < 4; ++p)
                acc[r] = __builtin_amdgcn_fdot2_f32_bf16(bf16x2v{wj[2 * p], wj[2 * p + 1]}, bf16x2v{xv[2 * p], xv[2 * p + 1]},
                                                         acc[r], false);
        }
    }
#pragma unroll
    for (int r = 0; r < MAXM; ++r)   // the lanes of each column: a half-wave, or the whole wave
        acc[r] = CPW == 2 ? half_wave_sum(acc[r]) : wave_sum_x(acc[r]);
    // lane hl = r of each column's lanes finishes row r of its column
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < MAXM; ++r)
        if (hl == r) v = acc[r];
    const int m = hl, n = col;
    if (m >= M || n >= a.N) return;
    if (a.bias) v += bias_raw;
    float rv = 0.f;
    if (has_res) {
        rv = res32 ? __uint_as_float(res_raw) : bf2f(__builtin_bit_cast(bf16, (unsigned short)res_raw));
        if (!(a.flags & CBW_EPI_RES_AFTER_ACT)) v += rv;
    }
    if (a.flags & CBW_EPI_RELU) v = fmaxf(v, 0.f);
    else if (a.flags & CBW_EPI_GELU) v = gelu_erf(v);
    if (has_res && (a.flags & CBW_EPI_RES_AFTER_ACT)) v += rv;
    if (a.flags & CBW_EPI_OUT_F32) {
        ((float*)a.y)[(int64_t)m * a.ldy + n] = v;
    } else {
        const bf16 o = f2bf(v);
        ((bf16*)a.y)[(int64_t)m * a.ldy + n] = o;
        if (a.kv_k && n >= a.kv_D) {
            const int64_t po = a.kv_pos ? (int64_t)a.kv_pos[a.kv_pos_rows ? m : 0] * a.kv_D : 0;
            bf16* dst = (n < 2 * a.kv_D ? a.kv_k + (n - a.kv_D) : a.kv_v + (n - 2 * a.kv_D)) + po;
            dst[(int64_t)m * a.kv_ld] = o;
        }
    }
}

}  // namespace

int cbw_gemv_waves(int K) {   // enough waves that each owns <= GV_BATCH k-steps (one burst of loads), at most 16
    const int ks = K / 32;
    int W = 1;
    while (W < 16 && (ks + W - 1) / W > GV_BATCH) W *= 2;
    return W;
}

namespace {
// the 16-row instantiations stage up to GD_LDS16 of rows: above the 64 KB default, raised once per kernel
template <auto KERNEL, int MAXM>
void dot_launch(dim3 grid, dim3 block, size_t lds, hipStream_t st, const GemvArgs& a) {
    if constexpr (MAXM > GD_MAXM) {
        static const bool once =
            hipFuncSetAttribute((const void*)KERNEL, hipFuncAttributeMaxDynamicSharedMemorySize, GD_LDS16) == hipSuccess;
        (void)once;
    }
    hipLaunchKernelGGL(KERNEL, grid, block, lds, st, a);
}

// rows 0..7 run the same arithmetic in either instantiation (each row's sums are independent of M and of the wave
// count), so a step over several windows' beams gives each window's rows the values a step over that window alone
// gives.  One column per wave for the K 5120 Linear (fc2, no LayerNorm); its 9..16-row rows staged in two K halves.
template <int NJ, int MAXM, int WV>
hipError_t launch_dot_m(const GemvArgs& a, size_t lds, hipStream_t st) {
    const dim3 block(WV * 64);
    const dim3 grid2((a.N + WV * 2 - 1) / (WV * 2)), grid1((a.N + WV - 1) / WV);
    if constexpr (NJ * 256 <= GV_LN_MAXK) {
        if (a.xf) {
            dot_launch<gemv_dot_kernel<true, NJ, 2, MAXM, 1, WV>, MAXM>(grid2, block, lds, st, a);
            return hipGetLastError();
        }
    }
    if (a.xf) return hipErrorInvalidValue;   // gemv_dot_wanted admits a LayerNorm prologue only for K <= 1280
    if constexpr (NJ == 20) {
        if constexpr (MAXM > GD_MAXM) {   // rows staged in two K halves
            const size_t lds2 = ((size_t)a.M * (a.K / 2) * 2 + 1023) / 1024 * 1024;
            dot_launch<gemv_dot_kernel<false, NJ, 1, MAXM, 2, WV>, MAXM>(grid1, block, lds2, st, a);
        } else {
            dot_launch<gemv_dot_kernel<false, NJ, 1, MAXM, 1, WV>, MAXM>(grid1, block, lds, st, a);
        }
        return hipGetLastError();
    }
    dot_launch<gemv_dot_kernel<false, NJ, 2, MAXM, 1, WV>, MAXM>(grid2, block, lds, st, a);
    return hipGetLastError();
}

template <int NJ>
hipError_t launch_dot(const GemvArgs& a, size_t lds, hipStream_t st) {
    if (a.M <= GD_MAXM) return launch_dot_m<NJ, GD_MAXM, 4>(a, lds, st);
    return launch_dot_m<NJ, 16, 8>(a, lds, st);   // eight computing waves for 9..16 rows
}

bool gemv_dot_wanted(const GemvArgs& a) {
    const int nj = a.K / 256;
    const bool nj_ok = nj == 3 || nj == 4 || nj == 5 || nj == 12 || nj == 16 || nj == 20;
    const size_t lds_max = a.M <= GD_MAXM ? 64 * 1024 : GD_LDS16;
    return a.M <= 16 && a.K % 256 == 0 && nj_ok && (size_t)a.M * (a.K + 8) * 2 <= lds_max &&
           (!a.xf || a.K <= GV_LN_MAXK) && a.ldx % 8 == 0;
}
}  // namespace

bool cbw_gemv_ln_ok(int M, int K) {
    return M >= 1 && M <= 16 && K % 32 == 0 && K <= GV_LN_MAXK && (size_t)M * (K + 8) * 2 <= GV_LN_LDS;
}

hipError_t cbw_gemv(const GemvArgs& a, hipStream_t st) {
    if (a.M < 1 || a.M > 16 || a.K % 32 || a.N % 4 || a.ldx % 8 || a.ldy % 4 || (a.res && a.res_ld % 4))
        return hipErrorInvalidValue;
    if (a.xf && (!a.ln_g || !a.ln_b || a.ldx % 4 || !cbw_gemv_ln_ok(a.M, a.K))) return hipErrorInvalidValue;
    if (a.kv_k && (!a.kv_v || a.kv_D % 4 || a.N != 3 * a.kv_D || a.kv_ld % 4 || (a.flags & CBW_EPI_OUT_F32)))
        return hipErrorInvalidValue;
    if (gemv_dot_wanted(a)) {
        // LayerNorm prologue: padded rows [M][K + 8]; else rows packed [M][K], DMA'd in whole 1 KB pieces
        const size_t lds = a.xf ? (size_t)a.M * (a.K + 8) * 2 : ((size_t)a.M * a.K * 2 + 1023) / 1024 * 1024;
        switch (a.K / 256) {
#define GD_CASE(NJ) \
    case NJ: return launch_dot<NJ>(a, lds, st);
            GD_CASE(3) GD_CASE(4) GD_CASE(5) GD_CASE(12) GD_CASE(16) GD_CASE(20)
#undef GD_CASE
            default: break;
        }
    }
    const int W = cbw_gemv_waves(a.K);
    const size_t lds = a.xf ? (size_t)a.M * (a.K + 8) * 2 : 0;
    if (a.xf) {
        if (W > 8) return hipErrorInvalidValue;
        hipLaunchKernelGGL(gemv_kernel<true>, dim3((a.N + 15) / 16), dim3(64 * W), lds, st, a);
    } else {
        hipLaunchKernelGGL(gemv_kernel<false>, dim3((a.N + 15) / 16), dim3(64 * W), 0, st, a);
    }
    return hipGetLastError();
}
