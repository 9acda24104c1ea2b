// Shared device helpers for the CB-Whisper gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CBW_DEV __device__ __forceinline__

CBW_DEV float bf2f(bf16 x) { return (float)x; }
CBW_DEV bf16 f2bf(float x) { return (bf16)x; }  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving)

CBW_DEV float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// __shfl_xor(v, O, 64) for O < 32 on a full wave without the ds_bpermute round trip: O = 1, 2 as DPP quad_perm
// ([1,0,3,2], [2,3,0,1]), O = 8 as DPP row_ror:8 (within a 16-lane row, lane i + 8 mod 16 = i ^ 8), O = 4, 16 as
// ds_swizzle (bit mode, xor within 32 lanes).  The same partner lane as the shuffle, so sums built from it are
// bit-identical to the shuffle versions.  Every lane of the wave must be active.
template <int O>
CBW_DEV float xor_lane(float v) {
    static_assert(O == 1 || O == 2 || O == 4 || O == 8 || O == 16, "xor_lane: O in {1, 2, 4, 8, 16}");
    const int x = __float_as_int(v);
    if constexpr (O == 1) return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));
    else if constexpr (O == 2) return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));
    else if constexpr (O == 8) return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false));
    else return __int_as_float(__builtin_amdgcn_ds_swizzle(x, 0x1F | (O << 10)));
}
// wave_sum / wave_max with the xor 16 .. 1 steps on xor_lane (full wave only): the same butterfly in the same order,
// so bit-identical to them
CBW_DEV float wave_sum_x(float v) {
    v += __shfl_xor(v, 32, 64);
    v += xor_lane<16>(v);
    v += xor_lane<8>(v);
    v += xor_lane<4>(v);
    v += xor_lane<2>(v);
    v += xor_lane<1>(v);
    return v;
}
CBW_DEV float wave_max_x(float v) {
    v = fmaxf(v, __shfl_xor(v, 32, 64));
    v = fmaxf(v, xor_lane<16>(v));
    v = fmaxf(v, xor_lane<8>(v));
    v = fmaxf(v, xor_lane<4>(v));
    v = fmaxf(v, xor_lane<2>(v));
    v = fmaxf(v, xor_lane<1>(v));
    return v;
}
// sum over each 32-lane half of the wave (the butterfly xor 16, 8, 4, 2, 1 of __shfl_xor, same order)
CBW_DEV float half_wave_sum(float v) {
    v += xor_lane<16>(v);
    v += xor_lane<8>(v);
    v += xor_lane<4>(v);
    v += xor_lane<2>(v);
    v += xor_lane<1>(v);
    return v;
}
CBW_DEV float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): blocks that share an XCD (b % 8 equal) get a contiguous
// range of tile ids so neighbouring tiles hit the same L2.
CBW_DEV int xcd_remap(int bid, int nwg) {
    if (nwg < 16) return bid;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
}

CBW_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
