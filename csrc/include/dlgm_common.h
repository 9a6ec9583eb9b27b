// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//   * wave64: all cross-lane reductions are written for 64 lanes (never 32);
//   * bf16 is clang's native __bf16 -- a plain (__bf16)f cast lowers to
//     v_cvt_pk_bf16_f32 on gfx950 which keeps NaN a NaN (needed by the NaN trap);
//   * memory-bound kernels move 16 B per lane per access (bf16x8 / float4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dlgm {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
// fp16 compute path (DeepSpeed "fp16" block): the same kernels instantiated on _Float16
typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef short short8 __attribute__((ext_vector_type(8)));
typedef short short4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x = NWAVES*64. `red` must hold NWAVES floats.
template <int NWAVES>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NWAVES; ++i) t += red[i];
  __syncthreads();
  return t;
}

template <int NWAVES>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
#pragma unroll
  for (int i = 0; i < NWAVES; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

// 8-element vector of a 16-bit storage type
template <typename T> struct vec8;
template <> struct vec8<bf16> { typedef bf16x8 type; };
template <> struct vec8<f16> { typedef f16x8 type; };
template <typename T> using vec8_t = typename vec8<T>::type;
template <typename T> struct vec4;
template <> struct vec4<bf16> { typedef bf16x4 type; };
template <> struct vec4<f16> { typedef f16x4 type; };
template <> struct vec4<float> { typedef f32x4 type; };
template <typename T> using vec4_t = typename vec4<T>::type;

template <typename T>
__device__ __forceinline__ f32x8 load8f(const T* p) {
  vec8_t<T> v = *reinterpret_cast<const vec8_t<T>*>(p);
  return __builtin_convertvector(v, f32x8);
}

template <typename T>
__device__ __forceinline__ void store8f(T* p, f32x8 v) {
  *reinterpret_cast<vec8_t<T>*>(p) = __builtin_convertvector(v, vec8_t<T>);
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

}  // namespace dlgm

#define DLGM_CHECK_HIP(expr)                                                   \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    TORCH_CHECK(_e == hipSuccess, "HIP error ", hipGetErrorString(_e), " at ", \
                __FILE__, ":", __LINE__);                                      \
  } while (0)

// Host: run `...` with T = the 16-bit device type of scalar type `st` (bf16, or fp16 for the fp16 path).
#define DLGM_DISPATCH_16(st, T, ...)                                                        \
  do {                                                                                     \
    if ((st) == at::kHalf) {                                                               \
      using T = dlgm::f16;                                                                 \
      __VA_ARGS__;                                                                         \
    } else {                                                                               \
      TORCH_CHECK((st) == at::kBFloat16, "expected a bf16 or fp16 tensor, got ", (st));    \
      using T = dlgm::bf16;                                                                \
      __VA_ARGS__;                                                                         \
    }                                                                                      \
  } while (0)

#define DLGM_IS16(t) ((t).scalar_type() == at::kBFloat16 || (t).scalar_type() == at::kHalf)
