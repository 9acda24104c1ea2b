// Row-stationary streaming 1x1 convolution for the HBM-bound ResNet-50 expand convs (gfx950).
//
// Serves the 1x1 stride-1 convs with a short reduction (K = Cin + Cin2 in {128, 256, 384, 512}) and a wide
// output: the identity-residual expand convs of stages 2 and 3 (HF ResNetBottleNeckLayer's last
// ResNetConvLayer + identity shortcut + ReLU, efficient_kws/resnet.py:51-58) and the stage-1 / stage-2
// first-block expand with the shortcut 1x1 conv folded in as a second K-source (ConvArgs::x2).  At LEF
// sizes these layers move 1-2 KB per output pixel (residual in, output out) against only K x Cout
// MACs, so they are HBM-bound (arithmetic intensity 57-116 FLOP/B for the identity expands).
//
// Design (why not a tile GEMM): a 128x128 tile kernel re-reads its A rows once per N-tile and its weight
// tile once per M-tile through L2, and must hide the residual's HBM latency inside one tile's short
// K loop.  Here the weights are STATIONARY in LDS and the rows in REGISTERS:
//   * each workgroup (one per CU, persistent) loads an N-slice of the folded weights W[n][k] (<= 128 KB,
//     XOR-swizzled 16-byte chunks) into LDS once, plus its bias slice;
//   * each wave is an independent streamer (no barrier after the setup): it takes a 32-pixel unit,
//     loads the unit's activation rows (32 x K bf16) straight into VGPRs as MFMA B-fragments, then
//     walks the slice in 64-channel steps: 4 x 2 x (K/32) mfma_f32_16x16x32_bf16 per step with the
//     weight fragments read from LDS by ds_read_b128, epilogue bias + residual + ReLU from the
//     accumulators, 8-byte stores;
//   * the residual of step s+2 is issued right after step s's epilogue (two steps in flight), so
//     every wave keeps ~8 KB of HBM reads outstanding besides its stores; 8-12 waves per CU do the
//     rest of the latency hiding;
//   * the output channels of a step are permuted across the MFMA fragments (perm_row) so that a lane
//     ends with 8 contiguous channels per fragment pair: residual loads and output stores are 16 bytes
//     per lane, 64 contiguous bytes per pixel per wave-instruction;
//   * when the weights need several slices (stage 3: 512 KB -> 4 x 128 KB), the workgroups of one
//     row group sit on the same XCD (blockIdx % 8) and walk the same units in the same order, so the
//     rows are fetched from HBM once and re-read from that XCD's L2.
// MFMAs run transposed (C^T = W . X^T): the pixel sits on the lane (fr), the channel on the register.
#include "cbw_common.h"
#include "cbw_kernels.h"

typedef int cs_i32x4 __attribute__((ext_vector_type(4)));
// raw buffer load / store (LLVM intrinsics by asm label): 32-bit offsets against one descriptor; the
// hardware range check returns 0 for / drops out-of-range lanes
__device__ cs_i32x4 cs_raw_load(cs_i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ void cs_raw_store(cs_i32x4 vdata, cs_i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.v4i32");

namespace {

constexpr int CS_NSTEP = 64;            // output channels per step (4 fragments of 16)
constexpr int CS_WBYTES = 131072;       // weight slice budget in LDS
constexpr int CS_MAXSLICE = 1024;       // bias slots

CBW_DEV cs_i32x4 cs_rsrc(const void* base, uint32_t bytes) {
    const uint64_t p = (uint64_t)base;
    cs_i32x4 r{(int)(uint32_t)p, (int)(uint32_t)(p >> 32), (int)bytes, 0x00020000};
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = __builtin_amdgcn_readfirstlane(r[q]);
    return r;
}
CBW_DEV cs_i32x4 cs_load(cs_i32x4 rsrc, int voff, int soff) { return cs_raw_load(rsrc, voff, soff, 0); }
CBW_DEV void cs_store(cs_i32x4 v, cs_i32x4 rsrc, int voff, int soff) { cs_raw_store(v, rsrc, voff, soff, 0); }

CBW_DEV int cs_off(int row, int chunk, int pitch) { return row * pitch + ((chunk ^ (row & 15)) << 4); }

// Output-channel permutation of a 64-channel step: MFMA fragment c (0..3), fragment row i = 4 fq + q
// computes channel 32 (c >> 1) + 8 fq + 4 (c & 1) + q, so lane (fr, fq) ends with 8 contiguous
// channels per fragment pair.  LDS weight row 16 c + i of a step holds that channel's weights.
CBW_DEV int perm_row(int r) {
    const int st = r & ~63, c = (r >> 4) & 3, i = r & 15;
    return st + 32 * (c >> 1) + 8 * (i >> 2) + 4 * (c & 1) + (i & 3);
}

// KS = K / 32 (k-steps of one MFMA); WAVES = waves per workgroup (register budget: 512 / (WAVES / 4));
// RD = residual steps in flight; PF = 16-pixel fragments per wave unit; PN = prefetch the next unit's rows
template <int KS, int WAVES, int RD, int PF, int PN>
__global__ __launch_bounds__(WAVES * 64, 1) void conv_stream_kernel(ConvArgs a, int nslice, int slice_n, int exp) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int K = KS * 32;
    constexpr int PITCH = K * 2;
    float* bias_s = (float*)(smem + slice_n * PITCH);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;

    // ---- workgroup -> (slice, row group): the nslice workgroups of a row group share an XCD
    const int G = gridDim.x;
    const int J = G / 8;                    // workgroups per XCD (G % 8 == 0, J % nslice == 0)
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int slice = j % nslice;
    const int rgs_per_xcd = J / nslice;
    const int rg = xcd * rgs_per_xcd + j / nslice;
    const int nrg = G / nslice;
    const int n_lo = slice * slice_n;

    // ---- setup: weight slice + bias slice -> LDS
    const bf16* __restrict__ Wt = (const bf16*)a.w;
    constexpr int CPR = K / 8;              // 16-byte chunks per weight row
    for (int e = tid; e < slice_n * CPR; e += WAVES * 64) {
        const int r = e / CPR, c = e - r * CPR;
        *(bf16x8*)(smem + cs_off(r, c, PITCH)) = *(const bf16x8*)(Wt + (int64_t)(n_lo + perm_row(r)) * K + c * 8);
    }
    for (int c = tid; c < slice_n; c += WAVES * 64) bias_s[c] = a.bias ? a.bias[n_lo + c] : 0.f;
    __syncthreads();

    const int M = a.M, Cin = a.Cin, Cin2 = a.x2 ? a.Cin2 : 0;
    const int HoWo = a.Ho * a.Wo, Wo = a.Wo;
    const bool relu = a.flags & CBW_EPI_RELU;
    const bool has_res = a.res != nullptr;
    const int nsteps = slice_n / CS_NSTEP;
    const int units = (M + (PF * 16) - 1) / (PF * 16);
    // buffer descriptors: 32-bit per-lane offsets, wave-uniform channel offsets in soffset; rows past M
    // get an offset past num_records (loads return 0, stores are dropped)
    const cs_i32x4 xr = cs_rsrc(a.x, (uint32_t)((int64_t)M * Cin * 2));
    const cs_i32x4 x2r = cs_rsrc(a.x2 ? a.x2 : a.x, a.x2 ? (uint32_t)((int64_t)a.N * a.H2 * a.W2 * Cin2 * 2) : 0u);
    const cs_i32x4 rr = cs_rsrc(has_res ? a.res : a.y, has_res ? (uint32_t)((int64_t)M * a.res_ld * 2) : 0u);
    const cs_i32x4 yr = cs_rsrc(a.y, (uint32_t)((int64_t)M * a.y_ld * 2));
    constexpr int OOR = 0x7ffffff0;

    // ---- a unit's rows -> B fragments (lane: pixel fr of fragment pf, k = 32 ks + 8 fq ..)
    auto load_rows = [&](int u, bf16x8 (&xv)[PF][KS], int (&ro)[PF], int (&yo)[PF]) {
#pragma unroll
        for (int pf = 0; pf < PF; ++pf) {
            const int p = u * (PF * 16) + pf * 16 + fr;
            const bool ok = p < M;
            const int xo = ok ? p * Cin * 2 + fq * 16 : OOR;
            int x2o = OOR;
            if (Cin2 && ok) {
                const int nn = p / HoWo, rem = p - nn * HoWo;
                const int oh = rem / Wo, ow = rem - oh * Wo;
                x2o = ((nn * a.H2 + oh * a.s2) * a.W2 + ow * a.s2) * Cin2 * 2 + fq * 16;
            }
            ro[pf] = ok ? p * a.res_ld * 2 + fq * 16 : OOR;
            yo[pf] = ok ? p * a.y_ld * 2 + fq * 16 : OOR;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const int k = ks * 32;
                const cs_i32x4 v = k < Cin ? cs_load(xr, xo, k * 2) : cs_load(x2r, x2o, (k - Cin) * 2);
                xv[pf][ks] = __builtin_bit_cast(bf16x8, v);
            }
        }
    };
    const int ustride = nrg * WAVES;
    int roff[PF], yoff[PF], roffn[PF], yoffn[PF];
    bf16x8 xf[PF][KS], xn[PF][KS];
    int u = rg * WAVES + wid;
    if (PN && u < units) load_rows(u, xn, roffn, yoffn);
    for (; u < units; u += ustride) {
        if (PN) {   // this unit's rows were issued during the previous unit's last steps
#pragma unroll
            for (int pf = 0; pf < PF; ++pf) {
                roff[pf] = roffn[pf];
                yoff[pf] = yoffn[pf];
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) xf[pf][ks] = xn[pf][ks];
            }
        } else {
            load_rows(u, xf, roff, yoff);
        }
        // ---- residual ring: steps s .. s + RD - 1 in flight.  Lane (fr, fq) owns channels
        // 32 h + 8 fq .. + 7 (h = 0, 1) of each 64-channel step: two 16-byte loads / stores per pixel
        // fragment, each wave-instruction covering 16 pixels x 64 contiguous bytes.
        cs_i32x4 res[RD][PF][2];
        auto load_res = [&](cs_i32x4 (&dst)[PF][2], int s) {
#pragma unroll
            for (int pf = 0; pf < PF; ++pf)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    dst[pf][h] = (exp & 1) ? cs_i32x4{0, 0, 0, 0}
                                           : cs_load(rr, roff[pf], (n_lo + s * CS_NSTEP + h * 32) * 2);
        };
        if (has_res) {
#pragma unroll
            for (int r = 0; r < RD; ++r)
                if (r < nsteps) load_res(res[r], r);
        }
        auto step = [&](cs_i32x4 (&rs)[PF][2], int s) {
            f32x4 acc[PF][4];
#pragma unroll
            for (int pf = 0; pf < PF; ++pf)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[pf][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                bf16x8 wf[4];
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    wf[c] = *(const bf16x8*)(smem + cs_off(s * CS_NSTEP + c * 16 + fr, ks * 4 + fq, PITCH));
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int pf = 0; pf < PF; ++pf)
                        acc[pf][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], xf[pf][ks], acc[pf][c], 0, 0, 0);
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int nl = s * CS_NSTEP + h * 32 + fq * 8;
                const f32x4 bv0 = *(const f32x4*)(bias_s + nl), bv1 = *(const f32x4*)(bias_s + nl + 4);
#pragma unroll
                for (int pf = 0; pf < PF; ++pf) {
                    float v[8];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        v[q] = acc[pf][2 * h][q] + bv0[q];
                        v[4 + q] = acc[pf][2 * h + 1][q] + bv1[q];
                    }
                    if (has_res) {
                        const bf16x8 rv = __builtin_bit_cast(bf16x8, rs[pf][h]);
#pragma unroll
                        for (int q = 0; q < 8; ++q) v[q] += bf2f(rv[q]);
                    }
                    bf16x8 o;
#pragma unroll
                    for (int q = 0; q < 8; ++q) o[q] = f2bf(relu ? fmaxf(v[q], 0.f) : v[q]);
                    const int yo = (exp & 2) ? (v[0] == 12345.f ? yoff[pf] : OOR) : yoff[pf];
                    cs_store(__builtin_bit_cast(cs_i32x4, o), yr, yo, (n_lo + s * CS_NSTEP + h * 32) * 2);
                }
            }
            if (has_res && s + RD < nsteps) load_res(rs, s + RD);
        };
        for (int s = 0; s < nsteps; s += RD) {   // nsteps % RD == 0 (slice_n % 128 == 0)
            // PN: the next unit's rows go out with the last RD steps (after their residual loads, so
            // waiting for those never waits for the prefetch)
            if (PN && s + RD >= nsteps && u + ustride < units) load_rows(u + ustride, xn, roffn, yoffn);
#pragma unroll
            for (int r = 0; r < RD; ++r) step(res[r], s + r);
        }
    }
}

int num_cus_cs() {   // the persistent grid; CBW_CS_CUS=N (A/B) sizes it for N CUs, leaving the rest to the other streams
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        const char* e = getenv("CBW_CS_CUS");
        if (e && atoi(e) > 0) n = std::min(n, atoi(e));
    }
    return n;
}

int cs_exp() {   // CBW_CS_EXP diagnostic builds: 1 no residual loads, 2 no stores (wrong results)
    const char* e = getenv("CBW_CS_EXP");
    return e ? atoi(e) : 0;
}

int stream_prefetch() {   // CBW_CS_PREFETCH: -1 policy (default), 0 off, 1 on wherever it fits the registers
    const char* e = getenv("CBW_CS_PREFETCH");
    return e ? atoi(e) : -1;
}

// K 512 on the streaming kernel (16-pixel units, 8 waves; CBW_CS_K512=0 keeps the tile kernels).
// tools/layer_bench.py, LEF chunk of 500: stage-2 reduce 512 -> 128 140.7 -> 120.5 us, stage-3 first
// reduce 512 -> 256 227.0 -> 183.9 us, stage-4 identity expand 512 -> 2048 + res 163.4 -> 120.7 us
int stream_k512() {
    const char* e = getenv("CBW_CS_K512");
    return e ? atoi(e) : 1;
}

int stream_mode() {   // CBW_CONV_STREAM=0 keeps these convs on the tile kernels (A/B experiments)
    const char* e = getenv("CBW_CONV_STREAM");
    return e ? atoi(e) : 1;
}

// the weight slice: the largest divisor of Cout that is a multiple of 128 channels and fits the budget
int slice_channels(int cout, int ktot) {
    for (int nsl = 1; nsl <= cout / 128; ++nsl) {
        if (cout % nsl) continue;
        const int sn = cout / nsl;
        if (sn % 128 == 0 && sn <= CS_MAXSLICE && (int64_t)sn * ktot * 2 <= CS_WBYTES) return sn;
    }
    return 0;
}

}  // namespace

thread_local int cbw_cs_grid_cus = 0;

bool cbw_conv_stream_supported(const ConvArgs& a) {
    const int ktot = a.Cin + (a.x2 ? a.Cin2 : 0);
    if (a.KH != 1 || a.KW != 1 || a.sh != 1 || a.sw != 1 || a.ph != 0 || a.pw != 0) return false;
    if (ktot != 128 && ktot != 256 && ktot != 384 && !(ktot == 512 && stream_k512())) return false;
    if (a.Cin % 32 || (a.x2 && a.Cin2 % 32)) return false;
    if (a.flags & ~CBW_EPI_RELU) return false;                   // bf16 residual / output, ReLU or none
    if (a.res && a.res_ld % 4) return false;
    if (a.y_ld % 4 || a.M <= 0) return false;
    const int64_t lim = 0x7ffffff0LL - 4096;   // 32-bit buffer offsets, out-of-range marker above
    if ((int64_t)a.M * a.y_ld * 2 >= lim || (int64_t)a.M * a.Cin * 2 >= lim) return false;
    if (a.res && (int64_t)a.M * a.res_ld * 2 >= lim) return false;
    if (a.x2 && (int64_t)a.N * a.H2 * a.W2 * a.Cin2 * 2 >= lim) return false;
    return slice_channels(a.Cout, ktot) > 0;
}

// policy: every supported conv -- at LEF sizes the identity expands (stage 2: 274 -> 244 us, stage 3: 182 ->
// 137 us), the folded-shortcut expands of stages 1-2 and the stage-2 first reduce (307 -> 284 us)
bool cbw_conv_stream_wanted(const ConvArgs& a) {
    return stream_mode() != 0 && cbw_conv_stream_supported(a);
}

hipError_t cbw_conv_stream(const ConvArgs& a, hipStream_t st) {
    if (!cbw_conv_stream_supported(a)) return hipErrorNotSupported;
    const int ktot = a.Cin + (a.x2 ? a.Cin2 : 0);
    const int sn = slice_channels(a.Cout, ktot);
    const int nslice = a.Cout / sn;
    const int cus = cbw_cs_grid_cus > 0 ? std::min(num_cus_cs(), cbw_cs_grid_cus) : num_cus_cs();
    const int G = 8 * nslice * std::max(1, cus / (8 * nslice));
    const size_t lds = (size_t)sn * ktot * 2 + (size_t)sn * 4;
    // (tools/layer_bench.py, LEF chunk of 500: K 128 -- 12 waves, 2 residual steps in flight 244 us vs
    // 16 waves, 1 step 256 us; K 256 -- 12 waves, 1 step 137 us vs 8 waves, 2 steps 143 us; 16-pixel units
    // with 16 waves: within 2 % at K 128, 6 % slower at K 256)
    // next-unit row prefetch (tools/layer_bench.py, LEF chunk of 500, LB_VAR=CBW_CS_PREFETCH): K 128 on 8 waves
    // 243.6 -> 237.6 us (stage-2 expand); K 256 on 8 waves 283.9 -> 273.5 us without a residual (stage-2 first
    // reduce) but 136.7 -> 142.5 us with one (stage-3 expand: the 12-wave residual latency hiding wins)
    const int pf = stream_prefetch();
    const int pn = pf >= 0 ? pf : (ktot == 128 || (ktot == 256 && !a.res));
#define CS_LAUNCH(KS, WAVES, RD, PFD, PN)                                                                               \
    do {                                                                                                           \
        cbw_last_conv_kernel = "conv_stream_kernel<" #KS ", " #WAVES ", " #RD ", " #PFD ", " #PN ">";                \
        hipLaunchKernelGGL((conv_stream_kernel<KS, WAVES, RD, PFD, PN>), dim3(G), dim3(WAVES * 64), lds, st, a,       \
                           nslice, sn, cs_exp());                                                                  \
    } while (0)
    switch (ktot) {
        case 128:
            if (pn) CS_LAUNCH(4, 8, 2, 2, 1);
            else CS_LAUNCH(4, 12, 2, 2, 0);
            break;
        case 256:
            if (pn) CS_LAUNCH(8, 8, 1, 2, 1);
            else CS_LAUNCH(8, 12, 1, 2, 0);
            break;
        case 512:
            CS_LAUNCH(16, 8, 2, 1, 0);
            break;
        default:   // (K 384 with the prefetch: 244 VGPRs spilled)
            CS_LAUNCH(12, 8, 2, 2, 0);
            break;
    }
#undef CS_LAUNCH
    return hipGetLastError();
}
