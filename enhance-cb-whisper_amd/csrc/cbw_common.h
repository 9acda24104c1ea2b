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
