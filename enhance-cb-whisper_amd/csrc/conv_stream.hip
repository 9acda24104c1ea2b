// Row-stationary streaming 1x1 convolution for the HBM-bound ResNet-50 expand convs (gfx950).
//
// Serves the 1x1 stride-1 convs with a short reduction (K = Cin + Cin2 in {128, 256, 384}) and a wide
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

namespace {

constexpr int CS_PX = 32;               // pixels per wave unit (2 fragments of 16)
constexpr int CS_PF = CS_PX / 16;
constexpr int CS_NSTEP = 64;            // output channels per step (4 fragments of 16)
constexpr int CS_WBYTES = 131072;       // weight slice budget in LDS
constexpr int CS_MAXSLICE = 1024;       // bias slots

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

CBW_DEV int cs_off(int row, int chunk, int pitch) { return row * pitch + ((chunk ^ (row & 15)) << 4); }

// Output-channel permutation of a 64-channel step: MFMA fragment c (0..3), fragment row i = 4 fq + q
// computes channel 32 (c >> 1) + 8 fq + 4 (c & 1) + q, so lane (fr, fq) ends with 8 contiguous
// channels per fragment pair.  LDS weight row 16 c + i of a step holds that channel's weights.
CBW_DEV int perm_row(int r) {
    const int st = r & ~63, c = (r >> 4) & 3, i = r & 15;
    return st + 32 * (c >> 1) + 8 * (i >> 2) + 4 * (c & 1) + (i & 3);
}

// KS = K / 32 (k-steps of one MFMA); WAVES = waves per workgroup (register budget: 512 / (WAVES / 4))
template <int KS, int WAVES>
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

    const bf16* __restrict__ X = (const bf16*)a.x;
    const bf16* __restrict__ X2 = (const bf16*)a.x2;
    const bf16* __restrict__ R = (const bf16*)a.res;
    bf16* __restrict__ Y = (bf16*)a.y;
    const int M = a.M, Cin = a.Cin, Cin2 = a.x2 ? a.Cin2 : 0;
    const int HoWo = a.Ho * a.Wo, Wo = a.Wo;
    const int res_ld = a.res_ld, y_ld = a.y_ld;
    const bool relu = a.flags & CBW_EPI_RELU;
    const bool has_res = R != nullptr;
    const int nsteps = slice_n / CS_NSTEP;
    const int units = (M + CS_PX - 1) / CS_PX;

    for (int u = rg * WAVES + wid; u < units; u += nrg * WAVES) {
        // ---- this unit's rows -> B fragments (lane: pixel fr of fragment pf, k = 32 ks + 8 fq ..)
        int prow[CS_PF];
        bool pok[CS_PF];
        bf16x8 xf[CS_PF][KS];
#pragma unroll
        for (int pf = 0; pf < CS_PF; ++pf) {
            const int p = u * CS_PX + pf * 16 + fr;
            pok[pf] = p < M;
            prow[pf] = pok[pf] ? p : M - 1;
            const bf16* xr = X + (int64_t)prow[pf] * Cin + fq * 8;
            const bf16* xr2 = X2;
            if (Cin2) {
                const int nn = prow[pf] / HoWo, rem = prow[pf] - nn * HoWo;
                const int oh = rem / Wo, ow = rem - oh * Wo;
                xr2 = X2 + (((int64_t)nn * a.H2 + oh * a.s2) * a.W2 + ow * a.s2) * Cin2 + fq * 8;
            }
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const int k = ks * 32;
                xf[pf][ks] = k < Cin ? *(const bf16x8*)(xr + k) : *(const bf16x8*)(xr2 + (k - Cin));
            }
        }
        // ---- residual ring: steps s and s+1 in flight.  Lane (fr, fq) owns channels
        // 32 h + 8 fq .. + 7 (h = 0, 1) of each 64-channel step: two 16-byte loads / stores per pixel
        // fragment, each wave-instruction covering 16 pixels x 64 contiguous bytes.
        u32x4 res[2][CS_PF][2];
        auto load_res = [&](u32x4 (&dst)[CS_PF][2], int s) {
#pragma unroll
            for (int pf = 0; pf < CS_PF; ++pf)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    dst[pf][h] = (exp & 1) ? u32x4{0u, 0u, 0u, 0u}
                                           : *(const u32x4*)(R + (int64_t)prow[pf] * res_ld + n_lo + s * CS_NSTEP +
                                                             h * 32 + fq * 8);
        };
        if (has_res) {
            load_res(res[0], 0);
            if (nsteps > 1) load_res(res[1], 1);
        }
        auto step = [&](u32x4 (&rs)[CS_PF][2], int s) {
            f32x4 acc[CS_PF][4];
#pragma unroll
            for (int pf = 0; pf < CS_PF; ++pf)
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
                    for (int pf = 0; pf < CS_PF; ++pf)
                        acc[pf][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[c], xf[pf][ks], acc[pf][c], 0, 0, 0);
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int nl = s * CS_NSTEP + h * 32 + fq * 8;
                const f32x4 bv0 = *(const f32x4*)(bias_s + nl), bv1 = *(const f32x4*)(bias_s + nl + 4);
#pragma unroll
                for (int pf = 0; pf < CS_PF; ++pf) {
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
                    const bool st = (exp & 2) ? (v[0] == 12345.f) : pok[pf];
                    if (st) *(bf16x8*)(Y + (int64_t)prow[pf] * y_ld + n_lo + nl) = o;
                }
            }
            if (has_res && s + 2 < nsteps) load_res(rs, s + 2);
        };
        for (int s = 0; s < nsteps; s += 2) {   // nsteps is even (slice_n % 128 == 0)
            step(res[0], s);
            step(res[1], s + 1);
        }
    }
}

int num_cus_cs() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    }
    return n;
}

int cs_exp() {   // CBW_CS_EXP diagnostic builds: 1 no residual loads, 2 no stores (wrong results)
    const char* e = getenv("CBW_CS_EXP");
    return e ? atoi(e) : 0;
}

int stream_mode() {   // CBW_CONV_STREAM: 0 never, 1 policy (default)
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

bool cbw_conv_stream_supported(const ConvArgs& a) {
    const int ktot = a.Cin + (a.x2 ? a.Cin2 : 0);
    if (a.KH != 1 || a.KW != 1 || a.sh != 1 || a.sw != 1 || a.ph != 0 || a.pw != 0) return false;
    if (ktot != 128 && ktot != 256 && ktot != 384) return false;
    if (a.Cin % 32 || (a.x2 && a.Cin2 % 32)) return false;
    if (a.flags & ~CBW_EPI_RELU) return false;                   // bf16 residual / output, ReLU or none
    if (a.res && a.res_ld % 4) return false;
    if (a.y_ld % 4 || a.M <= 0) return false;
    return slice_channels(a.Cout, ktot) > 0;
}

// policy: the HBM-bound expands -- identity residual with K <= 256, or a folded shortcut with K <= 384
bool cbw_conv_stream_wanted(const ConvArgs& a) {
    if (stream_mode() == 0 || !cbw_conv_stream_supported(a)) return false;
    return a.res != nullptr || a.x2 != nullptr;
}

hipError_t cbw_conv_stream(const ConvArgs& a, hipStream_t st) {
    if (!cbw_conv_stream_supported(a)) return hipErrorNotSupported;
    const int ktot = a.Cin + (a.x2 ? a.Cin2 : 0);
    const int sn = slice_channels(a.Cout, ktot);
    const int nslice = a.Cout / sn;
    const int cus = num_cus_cs();
    const int G = 8 * nslice * std::max(1, cus / (8 * nslice));
    const size_t lds = (size_t)sn * ktot * 2 + (size_t)sn * 4;
    switch (ktot) {
        case 128: hipLaunchKernelGGL((conv_stream_kernel<4, 12>), dim3(G), dim3(768), lds, st, a, nslice, sn, cs_exp()); break;
        case 256: hipLaunchKernelGGL((conv_stream_kernel<8, 8>), dim3(G), dim3(512), lds, st, a, nslice, sn, cs_exp()); break;
        default: hipLaunchKernelGGL((conv_stream_kernel<12, 8>), dim3(G), dim3(512), lds, st, a, nslice, sn, cs_exp()); break;
    }
    return hipGetLastError();
}
