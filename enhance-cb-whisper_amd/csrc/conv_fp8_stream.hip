// Row-stationary streaming 1x1 convolution on e4m3 operands: the fp8 tier's HBM-bound 1x1 convs (the identity
// expands of stages 2-4 with their residual, the stride-1 reduces; HF ResNetBottleNeckLayer as called by
// src/efficient_kws/resnet.py:51-58).  conv_stream.hip's design in bytes (tools: the 4-wave fp8 tile kernel ran
// these at 1.3 TB/s -- one K-stage per tile, nothing overlapping its load, MFMAs and epilogue):
//   * one persistent workgroup per CU holds an N-slice of the e4m3 weights [n][k] (<= 128 KB, XOR-swizzled
//     16-byte chunks) and the slice's alpha / bias in LDS;
//   * each wave streams 16-pixel fragments: the rows go straight from HBM into VGPRs as the B operand of
//     v_mfma_scale_f32_16x16x128_f8f6f4 (32 bytes per lane per k-step: channels 128 ks + 32 fq ..), the weight
//     fragments come from LDS, 64 output channels per step as 4 MFMA fragments;
//   * the channels of a step are permuted over the fragments so lane (fr, fq) ends with channels
//     16 fq .. 16 fq + 15 of pixel fr: residual loads and output stores are 16 bytes per lane (e4m3), 64
//     contiguous bytes per pixel per wave-instruction;
//   * residuals RD steps ahead; rows of the next unit loaded during the current unit's last steps (PN);
//     buffer descriptors with 32-bit offsets (out-of-range rows read 0, stores dropped).
#include <algorithm>
#include <cstdlib>

#include "cbw_common.h"
#include "cbw_kernels.h"

typedef int f8s_i32x4 __attribute__((ext_vector_type(4)));
__device__ f8s_i32x4 f8s_raw_load(f8s_i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ void f8s_raw_store(f8s_i32x4 vdata, f8s_i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.v4i32");

namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int FS_NSTEP = 64;         // output channels per step (4 fragments of 16)
constexpr int FS_WBYTES = 131072;    // weight slice budget in LDS
constexpr float FS_MAX = 448.f;

CBW_DEV f8s_i32x4 fs_rsrc(const void* base, uint32_t bytes) {
    const uint64_t p = (uint64_t)base;
    f8s_i32x4 r{(int)(uint32_t)p, (int)(uint32_t)(p >> 32), (int)bytes, 0x00020000};
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = __builtin_amdgcn_readfirstlane(r[q]);
    return r;
}

// 16-byte chunk `chunk` of weight row `row` (pitch bytes = K): chunks XOR-swizzled by the row within the row's
// min(K / 16, 16) chunks
CBW_DEV int fs_off(int row, int chunk, int pitch) {
    const int m = (pitch >> 4) < 16 ? (pitch >> 4) - 1 : 15;
    return row * pitch + ((chunk ^ (row & m)) << 4);
}

// step row r (fragment c = (r >> 4) & 3, fragment row i = r & 15) computes channel 16 (i >> 2) + 4 c + (i & 3):
// the C^T layout puts fragment row i = 4 fq + q on lane quarter fq, so lane (fr, fq) holds 16 fq .. 16 fq + 15
CBW_DEV int fs_perm(int r) {
    const int st = r & ~63, c = (r >> 4) & 3, i = r & 15;
    return st + 16 * (i >> 2) + 4 * c + (i & 3);
}

// KS = K / 128 (k-steps of one MFMA), WAVES per workgroup, RD residual steps in flight, PF 16-pixel fragments per
// unit, PN next-unit row prefetch
template <int KS, int WAVES, int RD, int PF, int PN>
__global__ __launch_bounds__(WAVES * 64, 1) void conv_fp8_stream_kernel(F8ConvArgs a, int nslice, int slice_n) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int K = KS * 128;
    constexpr int PITCH = K;
    float* alpha_s = (float*)(smem + slice_n * PITCH);
    float* bias_s = alpha_s + slice_n;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int fr = lane & 15, fq = lane >> 4;

    const int G = gridDim.x;
    const int J = G / 8;
    const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
    const int slice = j % nslice;
    const int rgs_per_xcd = J / nslice;
    const int rg = xcd * rgs_per_xcd + j / nslice;
    const int nrg = G / nslice;
    const int n_lo = slice * slice_n;

    constexpr int CPR = K / 16;
    for (int e = tid; e < slice_n * CPR; e += WAVES * 64) {
        const int r = e / CPR, c = e - r * CPR;
        *(f8s_i32x4*)(smem + fs_off(r, c, PITCH)) = *(const f8s_i32x4*)(a.w + (int64_t)(n_lo + fs_perm(r)) * K + c * 16);
    }
    for (int c = tid; c < slice_n; c += WAVES * 64) {
        alpha_s[c] = a.alpha[n_lo + c];
        bias_s[c] = a.bias[n_lo + c];
    }
    __syncthreads();

    const int M = a.M, Cout = a.Cout;
    const bool has_res = a.res != nullptr;
    const int nsteps = slice_n / FS_NSTEP;
    const int units = (M + PF * 16 - 1) / (PF * 16);
    const f8s_i32x4 xr = fs_rsrc(a.x, (uint32_t)((int64_t)M * K));
    const f8s_i32x4 rr = fs_rsrc(has_res ? (const void*)a.res : (const void*)a.x, has_res ? (uint32_t)((int64_t)M * Cout) : 0u);
    const int osz = a.out_bf16 ? 2 : 1;
    const f8s_i32x4 yr = fs_rsrc(a.y, (uint32_t)((int64_t)M * Cout * osz));
    constexpr int OOR = 0x7ffffff0;

    auto load_rows = [&](int u, i32x8 (&xv)[PF][KS], int (&po)[PF]) {
#pragma unroll
        for (int pf = 0; pf < PF; ++pf) {
            const int p = u * (PF * 16) + pf * 16 + fr;
            const bool ok = p < M;
            const int xo = ok ? p * K + fq * 32 : OOR;
            po[pf] = ok ? p : -1;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const f8s_i32x4 lo = f8s_raw_load(xr, xo, ks * 128, 0);
                const f8s_i32x4 hi = f8s_raw_load(xr, xo, ks * 128 + 16, 0);
                xv[pf][ks] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            }
        }
    };
    const int ustride = nrg * WAVES;
    int pix[PF], pixn[PF];
    i32x8 xf[PF][KS], xn[PF][KS];
    int u = rg * WAVES + wid;
    if (PN && u < units) load_rows(u, xn, pixn);
    for (; u < units; u += ustride) {
        if (PN) {
#pragma unroll
            for (int pf = 0; pf < PF; ++pf) {
                pix[pf] = pixn[pf];
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) xf[pf][ks] = xn[pf][ks];
            }
        } else {
            load_rows(u, xf, pix);
        }
        f8s_i32x4 res[RD][PF];
        auto load_res = [&](f8s_i32x4 (&dst)[PF], int s) {
#pragma unroll
            for (int pf = 0; pf < PF; ++pf)
                dst[pf] = f8s_raw_load(rr, pix[pf] >= 0 ? pix[pf] * Cout + fq * 16 : OOR, n_lo + s * FS_NSTEP, 0);
        };
        if (has_res) {
#pragma unroll
            for (int r = 0; r < RD; ++r)
                if (r < nsteps) load_res(res[r], r);
        }
        auto step = [&](f8s_i32x4 (&rs)[PF], int s) {
            f32x4 acc[PF][4];
#pragma unroll
            for (int pf = 0; pf < PF; ++pf)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[pf][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                i32x8 wf[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int row = s * FS_NSTEP + c * 16 + fr;
                    const f8s_i32x4 lo = *(const f8s_i32x4*)(smem + fs_off(row, ks * 8 + 2 * fq, PITCH));
                    const f8s_i32x4 hi = *(const f8s_i32x4*)(smem + fs_off(row, ks * 8 + 2 * fq + 1, PITCH));
                    wf[c] = i32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                }
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int pf = 0; pf < PF; ++pf)
                        acc[pf][c] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[c], xf[pf][ks], acc[pf][c], 0, 0,
                                                                                    0, 127, 0, 127);
            }
            const int nl = s * FS_NSTEP + fq * 16;   // lane's channels n_lo + nl .. + 15 (c -> 4 c + q)
#pragma unroll
            for (int pf = 0; pf < PF; ++pf) {
                float v[16];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const f32x4 al = *(const f32x4*)(alpha_s + nl + 4 * c), bb = *(const f32x4*)(bias_s + nl + 4 * c);
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[4 * c + q] = acc[pf][c][q] * al[q] + bb[q];
                }
                if (has_res) {
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const f32x2 r0 = __builtin_amdgcn_cvt_pk_f32_fp8(rs[pf][w], false);
                        const f32x2 r1 = __builtin_amdgcn_cvt_pk_f32_fp8(rs[pf][w], true);
                        v[4 * w] += r0[0] * a.res_scale; v[4 * w + 1] += r0[1] * a.res_scale;
                        v[4 * w + 2] += r1[0] * a.res_scale; v[4 * w + 3] += r1[1] * a.res_scale;
                    }
                }
                if (a.relu)
#pragma unroll
                    for (int q = 0; q < 16; ++q) v[q] = fmaxf(v[q], 0.f);
                const int yo = pix[pf] >= 0 ? pix[pf] * Cout * osz + fq * 16 * osz : OOR;
                if (a.out_bf16) {
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        bf16x8 o;
#pragma unroll
                        for (int q = 0; q < 8; ++q) o[q] = f2bf(v[8 * h + q]);
                        f8s_raw_store(__builtin_bit_cast(f8s_i32x4, o), yr, yo, (n_lo + s * FS_NSTEP) * 2 + h * 16, 0);
                    }
                } else {
                    f8s_i32x4 o;
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        float qv[4];
#pragma unroll
                        for (int q = 0; q < 4; ++q) qv[q] = fminf(fmaxf(v[4 * w + q] * a.y_inv_scale, -FS_MAX), FS_MAX);
                        int pk = __builtin_amdgcn_cvt_pk_fp8_f32(qv[0], qv[1], 0, false);
                        o[w] = __builtin_amdgcn_cvt_pk_fp8_f32(qv[2], qv[3], pk, true);
                    }
                    f8s_raw_store(o, yr, yo, n_lo + s * FS_NSTEP, 0);
                }
            }
            if (has_res && s + RD < nsteps) load_res(rs, s + RD);
        };
        for (int s = 0; s < nsteps; s += RD) {
            if (PN && s + RD >= nsteps && u + ustride < units) load_rows(u + ustride, xn, pixn);
#pragma unroll
            for (int r = 0; r < RD; ++r)
                if (s + r < nsteps) step(res[r], s + r);
        }
    }
}

int fs_num_cus() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    }
    return n;
}

int fs_slice(int cout, int k) {   // the largest divisor of Cout, a multiple of 64, within the LDS budget
    for (int nsl = 1; nsl <= cout / 64; ++nsl) {
        if (cout % nsl) continue;
        const int sn = cout / nsl;
        if (sn % 64 == 0 && (int64_t)sn * k <= FS_WBYTES) return sn;
    }
    return 0;
}

int fs_mode() {   // CBW_FP8_STREAM=0 keeps the fp8 1x1 convs on the tile kernels (A/B experiments)
    static const int m = [] {
        const char* e = getenv("CBW_FP8_STREAM");
        return e ? atoi(e) : 1;
    }();
    return m;
}

template <int KS, int WAVES, int RD, int PF, int PN>
hipError_t fs_launch(const F8ConvArgs& a, int G, int nslice, int sn, size_t lds, hipStream_t st) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)conv_fp8_stream_kernel<KS, WAVES, RD, PF, PN>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    static const std::string nm = kernel_name("conv_fp8_stream_kernel", {KS, WAVES, RD, PF, PN});
    cbw_last_conv_kernel = nm.c_str();
    hipLaunchKernelGGL((conv_fp8_stream_kernel<KS, WAVES, RD, PF, PN>), dim3(G), dim3(WAVES * 64), lds, st, a, nslice, sn);
    return hipGetLastError();
}

}  // namespace

bool cbw_conv_fp8_stream_supported(const F8ConvArgs& a) {
    if (!fs_mode() || a.KH != 1 || a.KW != 1 || a.sh != 1 || a.sw != 1 || a.M <= 0) return false;
    if (a.Cin != 128 && a.Cin != 256 && a.Cin != 512) return false;
    const int64_t lim = 0x7ffffff0LL - 4096;
    if ((int64_t)a.M * a.Cin >= lim || (int64_t)a.M * a.Cout * (a.out_bf16 ? 2 : 1) >= lim) return false;
    return fs_slice(a.Cout, a.Cin) > 0;
}

hipError_t cbw_conv_fp8_stream(const F8ConvArgs& a, hipStream_t st) {
    if (!cbw_conv_fp8_stream_supported(a)) return hipErrorNotSupported;
    const int sn = fs_slice(a.Cout, a.Cin);
    const int nslice = a.Cout / sn;
    const int cus = cbw_cs_grid_cus > 0 ? std::min(fs_num_cus(), cbw_cs_grid_cus) : fs_num_cus();
    const int G = 8 * nslice * std::max(1, cus / (8 * nslice));
    const size_t lds = (size_t)sn * a.Cin + (size_t)sn * 8;
    switch (a.Cin) {
        case 128: return fs_launch<1, 8, 2, 2, 1>(a, G, nslice, sn, lds, st);
        case 256: return fs_launch<2, 8, 2, 2, 1>(a, G, nslice, sn, lds, st);
        default: return fs_launch<4, 8, 2, 1, 0>(a, G, nslice, sn, lds, st);   // (PF 2: 70 VGPRs spilled)
    }
}
