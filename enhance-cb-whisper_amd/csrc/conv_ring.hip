// Persistent 8-wave implicit-GEMM convolution for the ResNet classifier convs (gfx950).
//
// One workgroup per CU walks its output tiles (BM = 256 pixels x BN = 128 channels) as ONE
// flattened stream of K-stages (BK = 64): a 3-slot LDS ring filled by global_load_lds keeps two
// stages in flight at every barrier -- also across tile boundaries, so the next tile's first stages
// land while the current tile finishes its MFMAs and epilogue.  Every wait is a counted
// s_waitcnt vmcnt(N) derived from a running count of the vector-memory ops the wave has issued
// (glds stages, output stores), never vmcnt(0) inside the stream, and the
// barrier is a raw s_barrier (cdna_hip_programming.md §5 "Pipelining across barriers").
//
// Serves the ResNet-50 1x1 convs with Cout % 128 == 0, short K and no residual (the first-block reduce
// convs, the stage-2 reduce, the expand convs with the folded shortcut as a second K-source) in place
// of the one-tile-per-block kernels of conv_igemm.hip (HF ResNetConvLayer / ResNetShortCut as run by
// efficient_kws/resnet.py:51-58).  Within a K-stage the first half's MFMAs run while the second
// half's fragments are read, and the next stage's glds issue sits between the two halves.
//
// Layout: 128-byte LDS rows (64 bf16 of K), 16-byte chunk index XOR ((row >> 1) & 7) applied on the
// glds SOURCE address (the LDS side of a glds is lane-linear); 8 waves as 4 (M) x 2 (N), each a
// 64 x 64 output tile of 4 x 4 mfma_f32_16x16x32_bf16, run transposed (C^T = W . X^T) so a lane
// ends with 4 consecutive channels of one pixel.  Epilogue straight from the accumulators: bias
// (from LDS), ReLU, bf16, raw buffer stores (rows past M dropped by the range
// check, so every wave issues the same number of stores and the counted waits stay exact).
#include "cbw_common.h"
#include "cbw_kernels.h"

typedef int ring_i32x2 __attribute__((ext_vector_type(2)));
typedef int ring_i32x4 __attribute__((ext_vector_type(4)));
__device__ void ring_store_v2i32(ring_i32x2 vdata, ring_i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.v2i32");

namespace {

constexpr int R_BM = 256, R_BN = 128, R_BK = 64, R_NS = 3;
constexpr int R_STAGE = (R_BM + R_BN) * 128;                 // 48 KB
constexpr int R_MAXC = 2048;                                 // bias slots in LDS
constexpr int R_LDS = R_NS * R_STAGE + R_MAXC * 4;           // 155648
static_assert(R_LDS <= 163840, "LDS budget");
constexpr int R_G = (R_BM + R_BN) * 128 / 16 / 512;          // glds per thread per stage: 6
constexpr int R_NST = 16;                                    // output stores per lane per tile

CBW_DEV int rswz(int r) { return (r >> 1) & 7; }

// s_waitcnt vmcnt(n) for a wave-uniform runtime n.  The counts that occur are sums of 6 (a glds
// stage) and 16 (stores); n is rounded DOWN to the nearest rung of the ladder
// (waiting for more ops than needed is always safe).
#define RING_VM(k) asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory")
CBW_DEV void wait_vm(int n) {
    if (n >= 38) { if (n >= 44) RING_VM(44); else RING_VM(38); }
    else if (n >= 22) { if (n >= 32) RING_VM(32); else if (n >= 28) RING_VM(28); else RING_VM(22); }
    else if (n >= 12) { if (n >= 16) RING_VM(16); else RING_VM(12); }
    else if (n >= 6) RING_VM(6);
    else RING_VM(0);
}
#undef RING_VM

CBW_DEV ring_i32x4 ring_rsrc(const void* base, uint32_t bytes) {
    const uint64_t p = (uint64_t)base;
    return ring_i32x4{(int)(uint32_t)p, (int)(uint32_t)(p >> 32), (int)bytes, 0x00020000};
}

template <int KH, int KW>
__global__ __launch_bounds__(512, 1) void conv_ring_kernel(ConvArgs a, int ntiles) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float* bias_s = (float*)(smem + R_NS * R_STAGE);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int fr = lane & 15, fq = lane >> 4;
    const int nt_n = a.Cout / R_BN;
    const bool dual = (KH * KW == 1) && a.x2 != nullptr;
    const int cin2 = dual ? a.Cin2 : 0;
    const int Ktot = KH * KW * a.Cin + cin2;
    const int csteps = a.Cin / R_BK;
    const int nsteps = KH * KW * csteps + cin2 / R_BK;
    const int HoWo = a.Ho * a.Wo;
    const int G = gridDim.x;
    const int my_tiles = (ntiles - (int)blockIdx.x + G - 1) / G;
    const int total = my_tiles * nsteps;
    if (total <= 0) return;
    const bool relu = a.flags & CBW_EPI_RELU;
    const bf16* __restrict__ X = (const bf16*)a.x;
    const bf16* __restrict__ X2 = (const bf16*)a.x2;
    const bf16* __restrict__ Wt = (const bf16*)a.w;
    const void* zero = a.zero;
    const int H = a.H, Wd = a.W, Cin = a.Cin, Cin2 = a.Cin2, H2 = a.H2, W2 = a.W2, s2 = a.s2;
    const int sh = a.sh, sw_ = a.sw, ph = a.ph, pw = a.pw, M = a.M, Wo = a.Wo;

    for (int c = tid; c < a.Cout; c += 512) bias_s[c] = a.bias ? a.bias[c] : 0.f;
    __syncthreads();

    // ---- issue cursor: gather state of the tile whose stages are being issued
    const int sub_r = lane >> 3, chunk = lane & 7;
    int64_t a_base[4], a_base2[4];
    int a_ih0[4], a_iw0[4];
    bool a_ok[4];
    const bf16* wrow[2];

    // ---- vector-memory op bookkeeping (wave-uniform): ops issued so far, and the count right
    // after each in-flight stage's glds (scalars: a dynamically indexed array would live in
    // scratch, i.e. more vector-memory ops) / after the residual loads
    int ops = 0, mark0 = 0, mark1 = 0, mark2 = 0;
    int iss = 0, iss_tile = 0, iss_s = 0;   // next stage to issue (flattened / tile / k-step)

    ring_i32x4 yr = ring_rsrc(a.y, (uint32_t)((int64_t)M * a.y_ld * 2));
#pragma unroll
    for (int q = 0; q < 4; ++q) yr[q] = __builtin_amdgcn_readfirstlane(yr[q]);
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    int tc = 0, sc = 0;   // tile / k-step of the stage being computed
    int m0 = 0, n0 = 0;
    bf16x8 av0[4], bv0[4], av1[4], bv1[4];
    // j = -2, -1: prologue (issue only)
    for (int j = -2; j < total; ++j) {
        if (j >= 0) {
            const int sl = j % R_NS;
            wait_vm(ops - (sl == 0 ? mark0 : (sl == 1 ? mark1 : mark2)));
            __builtin_amdgcn_s_barrier();
            if (sc == 0) {
                const int tile = xcd_remap(tc * G + (int)blockIdx.x, ntiles);
                m0 = (tile / nt_n) * R_BM;
                n0 = (tile % nt_n) * R_BN;
            }
            // first K-half: fragments, MFMAs interleaved with the second half's fragment reads; the next
            // stage's glds issue (address math) follows, then the second half
            const char* A = smem + (j % R_NS) * R_STAGE;
            const char* B = A + R_BM * 128;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int r = wn * 64 + jj * 16 + fr;
                bv0[jj] = *(const bf16x8*)(B + r * 128 + ((fq ^ rswz(r)) * 16));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = wm * 64 + i * 16 + fr;
                av0[i] = *(const bf16x8*)(A + r * 128 + ((fq ^ rswz(r)) * 16));
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv0[jj], av0[i], acc[i][jj], 0, 0, 0);
                __builtin_amdgcn_s_setprio(0);
                __builtin_amdgcn_sched_barrier(0);
                const int rb_ = wn * 64 + i * 16 + fr, ra_ = wm * 64 + i * 16 + fr;
                bv1[i] = *(const bf16x8*)(B + rb_ * 128 + (((4 + fq) ^ rswz(rb_)) * 16));
                av1[i] = *(const bf16x8*)(A + ra_ * 128 + (((4 + fq) ^ rswz(ra_)) * 16));
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (iss < total) {
            if (iss_s == 0) {   // new tile: per-lane gather rows
                const int tile = xcd_remap(iss_tile * G + (int)blockIdx.x, ntiles);
                const int im0 = (tile / nt_n) * R_BM, in0 = (tile % nt_n) * R_BN;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int r = (q * 8 + wid) * 8 + sub_r;
                    const int m = im0 + r;
                    a_ok[q] = m < M;
                    const int mm = a_ok[q] ? m : 0;
                    const int n = mm / HoWo, rem = mm - n * HoWo;
                    const int oh = rem / Wo, ow = rem - oh * Wo;
                    a_ih0[q] = oh * sh - ph;
                    a_iw0[q] = ow * sw_ - pw;
                    const int swc = (chunk ^ rswz(r)) * 8;
                    a_base[q] = (int64_t)n * H * Wd * Cin + swc;
                    a_base2[q] = dual ? (((int64_t)n * H2 + oh * s2) * W2 + ow * s2) * Cin2 + swc : 0;
                }
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int r = (q * 8 + wid) * 8 + sub_r;
                    wrow[q] = Wt + (int64_t)(in0 + r) * Ktot + ((chunk ^ rswz(r)) * 8);
                }
            }
            const int slot = iss % R_NS;
            const int tap = iss_s / csteps;
            const int c0 = (iss_s - tap * csteps) * R_BK;
            const int kh = tap / KW, kw = tap - kh * KW;
            char* As = smem + slot * R_STAGE;
            char* Bs = As + R_BM * 128;
            const bool second = dual && iss_s >= csteps;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rb = q * 8 + wid;
                const void* src;
                if constexpr (KH * KW == 1) {
                    const bf16* p1 = second ? X2 + a_base2[q] + (iss_s - csteps) * R_BK
                                            : X + a_base[q] + ((int64_t)a_ih0[q] * Wd + a_iw0[q]) * Cin + c0;
                    src = a_ok[q] ? (const void*)p1 : zero;
                } else {
                    const int ih = a_ih0[q] + kh, iw = a_iw0[q] + kw;
                    const bool ok = a_ok[q] && ih >= 0 && ih < H && iw >= 0 && iw < Wd;
                    src = ok ? (const void*)(X + a_base[q] + ((int64_t)ih * Wd + iw) * Cin + c0) : zero;
                }
                __builtin_amdgcn_global_load_lds(src, (void*)(As + rb * 1024), 16, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int rb = q * 8 + wid;
                __builtin_amdgcn_global_load_lds((const void*)(wrow[q] + (int64_t)iss_s * R_BK), (void*)(Bs + rb * 1024),
                                                 16, 0, 0);
            }
            ops += R_G;
            if (slot == 0) mark0 = ops;
            else if (slot == 1) mark1 = ops;
            else mark2 = ops;
            ++iss;
            if (++iss_s == nsteps) {
                iss_s = 0;
                ++iss_tile;
            }
        }
        if (j < 0) continue;

        // second K-half (its fragments were read under the first half's MFMAs)
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
                acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bv1[jj], av1[i], acc[i][jj], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);

        if (++sc == nsteps) {
            // ---- epilogue of tile tc
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int col = n0 + wn * 64 + jj * 16 + fq * 4;
                const f32x4 bb = *(const f32x4*)(bias_s + col);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int m = m0 + wm * 64 + i * 16 + fr;
                    float v[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) v[q] = acc[i][jj][q] + bb[q];
                    if (relu) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) v[q] = fmaxf(v[q], 0.f);
                    }
                    bf16x4 o;
#pragma unroll
                    for (int q = 0; q < 4; ++q) o[q] = f2bf(v[q]);
                    const int off = m < M ? (int)(((int64_t)m * a.y_ld + col) * 2) : (int)0x80000000;
                    ring_store_v2i32(__builtin_bit_cast(ring_i32x2, o), yr, off, 0, 0);
                }
            }
            ops += R_NST;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
            sc = 0;
            ++tc;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int ring_cus() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    }
    return n;
}

template <int KH, int KW>
hipError_t launch_ring(const ConvArgs& a, hipStream_t st) {
    const int ntiles = ((a.M + R_BM - 1) / R_BM) * (a.Cout / R_BN);
    const int G = std::min(ntiles, ring_cus());
    static const std::string nm = kernel_name("conv_ring_kernel", {KH, KW});
    cbw_last_conv_kernel = nm.c_str();
    hipLaunchKernelGGL((conv_ring_kernel<KH, KW>), dim3(G), dim3(512), R_LDS, st, a, ntiles);
    return hipGetLastError();
}

}  // namespace

bool cbw_conv_ring_supported(const ConvArgs& a) {
    if (a.Cout % R_BN || a.Cout > R_MAXC || a.Cin % R_BK || a.M <= 0) return false;
    if (a.flags & ~CBW_EPI_RELU) return false;   // bf16 output, ReLU or none
    if (a.res) return false;                     // identity-residual expands: conv_igemm_persist
    if (a.y_ld % 4 || (int64_t)a.M * a.y_ld * 2 >= 0x7fffffffLL) return false;
    if (a.x2 && (a.KH * a.KW != 1 || a.Cin2 % R_BK)) return false;
    return (a.KH == 1 && a.KW == 1) || (a.KH == 3 && a.KW == 3);
}

hipError_t cbw_conv_ring(const ConvArgs& a, hipStream_t st) {
    if (!cbw_conv_ring_supported(a)) return hipErrorNotSupported;
    if (a.KH == 1) return launch_ring<1, 1>(a, st);
    return launch_ring<3, 3>(a, st);
}
