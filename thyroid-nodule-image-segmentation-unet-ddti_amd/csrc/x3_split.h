// Exact three-way bf16 split of an f32 value, v = h + m + l (kernels_gemm_x3.hip header), with
// the range edges made explicit.  One source for the device passes (to_x3, bn_dz_x3, the ConvT
// epilogue into an x3 image) and the host test hook unet_x3_split_host (runtime.hip), which
// tests/test_lib_cpu.py checks against the NumPy restatement in tests/x3_split_ref.py; the GPU
// test tests/test_gpu_x3.py checks the device bits against the same restatement.
//
//   normal v:           h = rne(v), m = rne(v - h), l = rne(v - h - m); both differences are
//                       exact in f32 and h + m + l == v exactly (8 + 8 + 8 significand bits)
//   |v| >= 0x1.FFp127:  rne(v) would overflow to inf (bf16 max is 0x1.FEp127), so h takes the
//   (finite)            largest finite bf16 of v's sign instead; v - h is exact (Sterbenz) and
//                       the split stays exact
//   v = +-inf, NaN:     h = v, m = l = 0 (without this, m = inf - inf = NaN would turn an
//                       infinite activation into NaN; the f32 path propagates inf).  Caveat of
//                       the six-product MFMA sum: Ah * Bm with Ah = inf and a zero piece Bm is
//                       inf * 0 = NaN, so an infinite operand gives NaN wherever the other
//                       operand is exactly representable in fewer than 16 bits (the f32 path
//                       gives +-inf there; 0 * inf is NaN in both)
//   subnormal v / tiny: bf16 keeps f32's exponent range, but its subnormal quantum is 2^-133
//   pieces              against f32's 2^-149, so bits of v below 2^-133 are dropped: the split
//                       error is <= 2^-134 absolute (relative error <= 2^-24 for |v| >= 2^-110)
//
// The three products the x3 kernels drop (Am Bl, Al Bm, Al Bl) are bounded by
// |m| <= 2^-8 |a|, |l| <= 2^-16 |a|: 2^-24 + 2^-24 + 2^-32 <= ~2^-23 |a b| together.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define X3_BF16_OVF 0x1.FFp127f   // |v| >= this rounds to inf in bf16 (RNE)
#define X3_BF16_MAX 0x1.FEp127f   // largest finite bf16
#define X3_F32_MAX 0x1.FFFFFEp127f

__host__ __device__ __forceinline__ float x3_bf16_to_f32(uint16_t b) {
    return __builtin_bit_cast(float, (uint32_t)b << 16);
}

// bf16 round-to-nearest-even on the bit level (NaN stays a quiet NaN): the host conversion;
// the device uses the hardware conversion (v_cvt_pk_bf16_f32), whose bits the GPU test pins
// to the same rule
__host__ __device__ __forceinline__ uint16_t x3_rne_bits(float v) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// the split of v with the bf16 conversion `cvt` (float -> bf16 bits)
template <class Cvt>
__host__ __device__ __forceinline__ void x3_split(float v, Cvt cvt, uint16_t& h, uint16_t& m, uint16_t& l) {
    const float a = __builtin_fabsf(v);
    const bool huge = a >= X3_BF16_OVF && a <= X3_F32_MAX;
    h = cvt(huge ? __builtin_copysignf(X3_BF16_MAX, v) : v);
    float r1 = v - x3_bf16_to_f32(h);
    r1 = a <= X3_F32_MAX ? r1 : 0.f;  // +-inf, NaN: h carries v, m = l = 0
    m = cvt(r1);
    l = cvt(r1 - x3_bf16_to_f32(m));
}

__device__ __forceinline__ uint16_t x3_cvt_dev(float v) { return __builtin_bit_cast(uint16_t, (__bf16)v); }

struct X3CvtDev {
    __device__ __forceinline__ uint16_t operator()(float v) const { return x3_cvt_dev(v); }
};
struct X3CvtHost {
    __host__ __device__ __forceinline__ uint16_t operator()(float v) const { return x3_rne_bits(v); }
};
