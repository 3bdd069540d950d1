// wk_misc.hip -- device-side synthetic clip generator, normalize_mfcc, and the
// firmware's sample / frame front (record_task) and per-window CMVN (detect_task).
#include "wk_common.h"
#include "wk_kernels.h"

using namespace wk;

namespace {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// clamp(0.1*N(0,1), -1, 1) (+ 0.1*sin(2*pi*440 t / 16000)
// on odd clips); N(0,1) by Box-Muller on a counter hash of (seed, clip, sample).
// Same arithmetic as oracle/wk_oracle.py:synth_clips.
__global__ void wk_synth_kernel(uint32_t seed, int64_t first, int64_t count, int n, float* __restrict__ out) {
  const int64_t total = count * (int64_t)n;
  for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = idx / n;
    const uint32_t s = (uint32_t)(idx - c * n);
    const uint64_t clip = (uint64_t)(first + c);
    const uint32_t key = mix32(seed ^ (uint32_t)(clip * 0x9E3779B9ull));
    const uint32_t h1 = mix32(key ^ (s * 2u + 0x68E31DA4u));
    const uint32_t h2 = mix32(h1 ^ 0xB5297A4Du);
    const float u1 = ((float)(h1 >> 8) + 1.0f) * (1.0f / 16777216.0f);
    const float u2 = (float)(h2 >> 8) * (1.0f / 16777216.0f);
    const float r = sqrtf(-2.0f * logf(u1));
    const float gs = r * cosf(6.2831853071795865f * u2);
    float x = fminf(fmaxf(0.1f * gs, -1.0f), 1.0f);
    if (clip & 1) {
      const float ph = (float)((s * 440u) % 16000u) * (1.0f / 16000.0f);
      x += 0.1f * sinf(6.2831853071795865f * ph);
    }
    out[idx] = x;
  }
}

// normalize_mfcc (ml_models/src/extract_mfcc.py:47-88), one wave per row.
__global__ void wk_normalize_kernel(const float* __restrict__ in, float* __restrict__ out, int64_t rows, int n,
                                    int method) {
  const int lane = threadIdx.x & 63;
  const int64_t row = blockIdx.x * (int64_t)(blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* x = in + row * n;
  float* y = out + row * n;
  if (method == 0 || method == 2) {  // standardization / cmvn (identical in the reference)
    float s = 0.0f;
    for (int i = lane; i < n; i += 64) s += x[i];
    const float mean = wave_sum(s) / (float)n;
    float q = 0.0f;
    for (int i = lane; i < n; i += 64) {
      const float d = x[i] - mean;
      q = __builtin_fmaf(d, d, q);
    }
    float sd = sqrtf(wave_sum(q) / (float)(n - 1));
    sd = sd == 0.0f ? 1.0f : sd;
    for (int i = lane; i < n; i += 64) y[i] = (x[i] - mean) / (sd + 1e-8f);
  } else if (method == 1) {  // minmax
    float mn = INFINITY, mx = -INFINITY;
    for (int i = lane; i < n; i += 64) {
      mn = fminf(mn, x[i]);
      mx = fmaxf(mx, x[i]);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      mn = fminf(mn, __shfl_xor(mn, m, 64));
      mx = fmaxf(mx, __shfl_xor(mx, m, 64));
    }
    for (int i = lane; i < n; i += 64) y[i] = (x[i] - mn) / (mx - mn + 1e-8f);
  } else {
    for (int i = lane; i < n; i += 64) y[i] = x[i];
  }
}

// The firmware's int8 MFCC quantisation (record_task, esp_wake_word_detector.cpp:128-131):
// lroundf (half away from zero) then saturate to int8.
__device__ __forceinline__ float device_q(float v) { return fminf(fmaxf(__builtin_roundf(v), -128.0f), 127.0f); }
__device__ __forceinline__ float device_q(int8_t v) { return (float)v; }

// The firmware's per-window CMVN (detect_task, esp_wake_word_detector.cpp:179-211) over
// a stream of MFCC frames [n][13] (frame-major, as write_one_frame_mfcc_to_buffer
// stores them): window w is frames w .. w+62, oldest first (read_whole_mfcc_buffer,
// :21-29).  Per coefficient: mean over the 63 frames, POPULATION std (/63),
// (v - mean) / (std + 1e-8), lroundf, saturate to int8.  One thread per (window,
// coefficient), summing frame 0 .. 62 in the firmware's order with no FMA
// contraction, so the int8 results are bit-identical to the C loops (the sums of
// int8 values are exact in fp32; the variance sum, division and sqrt are
// IEEE-rounded in the same order).  Outputs: the device's int8 buffer [w][63][13]
// and/or the same values as float features [w][13][63] (wk_cnn's layout: the
// esp-dl model reads the frame-major buffer as its NWC input).
template <typename T>
__global__ void wk_device_cmvn_kernel(const T* __restrict__ frames, int64_t n_windows, int8_t* __restrict__ out_i8,
                                      float* __restrict__ out_f) {
#pragma clang fp contract(off)
  const int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (idx >= n_windows * 13) return;
  const int64_t w = idx / 13;
  const int dim = (int)(idx - w * 13);
  const T* x = frames + w * 13 + dim;
  float sum = 0.0f;
  for (int f = 0; f < 63; ++f) sum += device_q(x[f * 13]);
  const float mean = sum / 63.0f;
  float var = 0.0f;
  for (int f = 0; f < 63; ++f) {
    const float d = device_q(x[f * 13]) - mean;
    var += d * d;
  }
  const float sd = sqrtf(var / 63.0f);
  for (int f = 0; f < 63; ++f) {
    const float q = fminf(fmaxf(__builtin_roundf((device_q(x[f * 13]) - mean) / (sd + 1e-8f)), -128.0f), 127.0f);
    if (out_i8) out_i8[(w * 63 + f) * 13 + dim] = (int8_t)q;
    if (out_f) out_f[(w * 13 + dim) * 63 + f] = q;
  }
}

// The firmware record task's sample path (esp_wake_word_detector.cpp:102-121),
// integer-exact: 48 kHz TDM frames of 4 int16 channels (CH0 MIC-L, CH1 AEC
// reference, CH2 MIC-R, CH3 unused) -> mono
//   m = (int16_t)(((L << 6) + (AEC << 5) + (R << 6)) >> 7)   (:106-111)
// -- the int32 sum can exceed int16 (|L| = |R| = 32767 gives 40958) and the
// firmware's cast keeps the low 16 bits, so does this -- then the [1, 2, 1] / 4
// decimation to 16 kHz: out[j] = (int16_t)((m[3j] + 2 m[3j+1] + m[3j+2]) >> 2)
// (:114-121; >> on int32 is arithmetic, as on the ESP32).  Each thread makes
// two output samples from six TDM samples = 48 contiguous bytes, three 16-byte
// loads (HBM-bound byte work: 24 B in, 2 B out (+4 with the float copy) per
// output sample).  The float copy is x / 32768 (torchaudio.load's scale, what
// wk_forward applies to WK_DTYPE_I16).
__device__ __forceinline__ int32_t tdm_mono(uint2 q) {   // one TDM sample: 4 int16 channels in 8 bytes
  const int32_t l = (int16_t)(q.x & 0xFFFFu), aec = (int16_t)(q.x >> 16), r = (int16_t)(q.y & 0xFFFFu);
  return (int16_t)((l * 64 + aec * 32 + r * 64) >> 7);
}
__device__ __forceinline__ int16_t tdm_out(int32_t m0, int32_t m1, int32_t m2) {
  return (int16_t)((m0 + 2 * m1 + m2) >> 2);
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void wk_record_front_kernel(const u32x4* __restrict__ tdm, int64_t n_out,
                                                              int16_t* __restrict__ out16, float* __restrict__ outf) {
  const int64_t pair = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t j = 2 * pair;
  if (j >= n_out) return;
  int16_t o[2];
  if (j + 1 < n_out) {
    const u32x4 a = __builtin_nontemporal_load(tdm + 3 * pair);
    const u32x4 b = __builtin_nontemporal_load(tdm + 3 * pair + 1);
    const u32x4 c = __builtin_nontemporal_load(tdm + 3 * pair + 2);
    o[0] = tdm_out(tdm_mono(make_uint2(a.x, a.y)), tdm_mono(make_uint2(a.z, a.w)), tdm_mono(make_uint2(b.x, b.y)));
    o[1] = tdm_out(tdm_mono(make_uint2(b.z, b.w)), tdm_mono(make_uint2(c.x, c.y)), tdm_mono(make_uint2(c.z, c.w)));
    *reinterpret_cast<uint32_t*>(out16 + j) = (uint32_t)(uint16_t)o[0] | ((uint32_t)(uint16_t)o[1] << 16);
    if (outf) *reinterpret_cast<float2*>(outf + j) = make_float2(o[0] * (1.0f / 32768.0f), o[1] * (1.0f / 32768.0f));
  } else {   // odd tail: the last output sample alone (three 8-byte TDM samples)
    const uint2* q = reinterpret_cast<const uint2*>(tdm) + 3 * j;
    o[0] = tdm_out(tdm_mono(q[0]), tdm_mono(q[1]), tdm_mono(q[2]));
    out16[j] = o[0];
    if (outf) outf[j] = o[0] * (1.0f / 32768.0f);
  }
}

// record_task's int8 frame quantisation (:128-131): lroundf (half away from
// zero), saturate to [-128, 127].
__global__ __launch_bounds__(256) void wk_quantize_frames_kernel(const float* __restrict__ x, int64_t n,
                                                                 int8_t* __restrict__ q) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    q[i] = (int8_t)device_q(x[i]);
}

// Streaming ring ingest (wk_stream_push): ring samples [pos, pos + m) (mod
// cap, m <= cap) from the pinned host staging ring, read across PCIe, into
// both copies of the mirrored device ring.
__global__ __launch_bounds__(256) void wk_ring_ingest_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                             int64_t cap, int64_t pos, int64_t m) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = pos + i < cap ? pos + i : pos + i - cap;
    const float v = src[p];
    dst[p] = v;
    dst[p + cap] = v;
  }
}

}  // namespace

namespace wk {

hipError_t launch_ring_ingest(const float* src, float* dst, int64_t cap, int64_t pos, int64_t m, hipStream_t stream) {
  if (m <= 0) return hipSuccess;
  if (pos < 0 || pos >= cap || m > cap) return hipErrorInvalidValue;
  int64_t blocks = (m + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(wk_ring_ingest_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, src, dst, cap, pos, m);
  return hipGetLastError();
}

hipError_t launch_record_front(const int16_t* tdm, int64_t n_out, int16_t* out16, float* outf, hipStream_t stream) {
  if (n_out <= 0) return hipSuccess;
  const int64_t pairs = (n_out + 1) / 2;
  hipLaunchKernelGGL(wk_record_front_kernel, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const u32x4*>(tdm), n_out, out16, outf);
  return hipGetLastError();
}

hipError_t launch_quantize_frames(const float* x, int64_t n, int8_t* q, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(wk_quantize_frames_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, x, n, q);
  return hipGetLastError();
}

hipError_t launch_device_cmvn(const void* frames, bool int8_in, int64_t n_windows, int8_t* out_i8, float* out_f,
                              hipStream_t stream) {
  if (n_windows <= 0) return hipSuccess;
  const int64_t threads = n_windows * 13;
  const unsigned blocks = (unsigned)((threads + 255) / 256);
  if (int8_in)
    hipLaunchKernelGGL(wk_device_cmvn_kernel<int8_t>, dim3(blocks), dim3(256), 0, stream, (const int8_t*)frames,
                       n_windows, out_i8, out_f);
  else
    hipLaunchKernelGGL(wk_device_cmvn_kernel<float>, dim3(blocks), dim3(256), 0, stream, (const float*)frames,
                       n_windows, out_i8, out_f);
  return hipGetLastError();
}

hipError_t launch_synth(uint32_t seed, int64_t first, int64_t count, int n, float* out, hipStream_t stream) {
  const int64_t total = count * (int64_t)n;
  if (total == 0) return hipSuccess;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(wk_synth_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, seed, first, count, n, out);
  return hipGetLastError();
}

hipError_t launch_normalize(const float* in, float* out, int64_t batch, int n_coef, int n_time, int method,
                            hipStream_t stream) {
  const int64_t rows = batch * n_coef;
  if (rows == 0) return hipSuccess;
  const int64_t blocks = (rows + 3) / 4;
  hipLaunchKernelGGL(wk_normalize_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, in, out, rows, n_time,
                     method);
  return hipGetLastError();
}

}  // namespace wk
