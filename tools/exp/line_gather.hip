// EXPERIMENT (not product): the HBM floor of the lookup's exact access pattern. line_gather_kernel reads a list of
// 128-B lines (8 lanes x 16 B each, fully coalesced, many in flight) and folds them into one value per thread, so its
// time is what the memory system needs for exactly the lines one lookup must touch; write_stream_kernel writes the
// lookup's output bytes as a pure 16-B-per-lane stream.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void line_gather_kernel(const float4* __restrict__ base, const int64_t* __restrict__ lines,
                                                          long long n, float* __restrict__ sink) {
  float acc = 0.f;
  const long long nthreads = (long long)gridDim.x * blockDim.x;
  const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  // thread t handles piece (t & 7) of lines (t >> 3) + k * nthreads/8
#pragma unroll 4
  for (long long i = t0; i < n * 8; i += nthreads) {
    const float4 v = base[lines[i >> 3] * 8 + (i & 7)];
    acc += v.x + v.y + v.z + v.w;
  }
  sink[t0] = acc;
}

// each thread: 16 line indices loaded first, then 16 independent 16-B loads in flight
__global__ __launch_bounds__(256) void line_gather16_kernel(const float4* __restrict__ base, const int64_t* __restrict__ lines,
                                                            long long n, float* __restrict__ sink) {
  const long long nthreads = (long long)gridDim.x * blockDim.x;
  const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  for (long long i0 = t0; i0 < n * 8; i0 += nthreads * 16) {
    int64_t li[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const long long i = i0 + k * nthreads;
      li[k] = i < n * 8 ? lines[i >> 3] * 8 + (i & 7) : -1;
    }
    float4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = li[k] >= 0 ? base[li[k]] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
  }
  sink[t0] = acc;
}

__global__ __launch_bounds__(256) void read_stream_kernel(const float4* __restrict__ in, long long n4, float* __restrict__ sink) {
  const long long nthreads = (long long)gridDim.x * blockDim.x;
  const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
#pragma unroll 8
  for (long long i = t0; i < n4; i += nthreads) {
    const float4 v = in[i];
    acc += v.x + v.y + v.z + v.w;
  }
  sink[t0] = acc;
}

__global__ __launch_bounds__(256) void write_stream_kernel(float4* __restrict__ out, long long n4) {
  const long long nthreads = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += nthreads)
    out[i] = make_float4(1.f, 2.f, 3.f, (float)i);
}

extern "C" int exp_line_gather(const void* base, const void* lines, long long n, void* sink, int blocks, void* stream) {
  hipLaunchKernelGGL(line_gather_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float4*)base,
                     (const int64_t*)lines, n, (float*)sink);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
extern "C" int exp_write_stream(void* out, long long n4, int blocks, void* stream) {
  hipLaunchKernelGGL(write_stream_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (float4*)out, n4);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
extern "C" int exp_line_gather16(const void* base, const void* lines, long long n, void* sink, int blocks, void* stream) {
  hipLaunchKernelGGL(line_gather16_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float4*)base,
                     (const int64_t*)lines, n, (float*)sink);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
extern "C" int exp_read_stream(const void* in, long long n4, void* sink, int blocks, void* stream) {
  hipLaunchKernelGGL(read_stream_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const float4*)in, n4, (float*)sink);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
