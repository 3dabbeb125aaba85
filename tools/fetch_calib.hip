// FETCH_SIZE / WRITE_SIZE calibration for the access shapes the step kernels issue (dev tool).
//
// The step kernels read and write SoA state with one dword per lane per field (4 B/lane,
// coalesced over 64 consecutive envs).  The MI355X guide calibrates FETCH_SIZE only for
// 16 B/lane streaming reads (reports 1/2 of the bytes); this program streams a KNOWN byte count
// through each shape so that `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` runs give the
// factor bytes / (counter kB * 1024) per shape.  tools/pmc_summary.py applies the measured
// dword factor (profiles/fetch_calibration.json) instead of assuming the 16 B/lane one.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
// run:   rocprofv3 --pmc FETCH_SIZE --output-format csv -d DIR -o run -- tools/fetch_calib
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

// 4 B/lane coalesced dword loads, grid-stride; one float per thread written (small, known).
__global__ void read_dword(const float* __restrict__ a, size_t n, float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += a[i];
  out[blockIdx.x * (size_t)blockDim.x + threadIdx.x] = s;
}

// 16 B/lane coalesced dwordx4 loads (the guide's calibrated shape).
__global__ void read_dwordx4(const float4* __restrict__ a, size_t n4, float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  out[blockIdx.x * (size_t)blockDim.x + threadIdx.x] = s;
}

// SoA gather exactly as the step kernels lay it out: field f of env e at a[f * n_envs + e],
// one lane per env, NF fields read in turn (each a coalesced 256-B dword row per wave).
__global__ void read_soa(const float* __restrict__ a, int nf, int n_envs, float* __restrict__ out) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_envs) return;
  float s = 0.f;
  for (int f = 0; f < nf; ++f) s += a[(size_t)f * n_envs + e];
  out[e] = s;
}

// 4 B/lane coalesced dword stores.
__global__ void write_dword(float* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = (float)(i & 1023);
}

int main() {
  const size_t n = (size_t)1 << 28;  // 1 GiB of floats: 4x the 256 MiB Infinity Cache
  const int nf = 64, n_envs = (int)(n / nf);
  float *a, *b, *out;
  CHECK(hipMalloc(&a, n * 4));
  CHECK(hipMalloc(&b, n * 4));
  CHECK(hipMalloc(&out, (size_t)n_envs * 4));
  CHECK(hipMemset(a, 0, n * 4));
  const int grid = 256 * 8 * 4, block = 256;  // 8192 workgroups, grid-stride
  // a is re-written between reads so that every read starts from a cold-ish cache state
  write_dword<<<grid, block>>>(b, n);
  read_dword<<<grid, block>>>(a, n, out);
  write_dword<<<grid, block>>>(b, n);
  read_dwordx4<<<grid, block>>>((const float4*)a, n / 4, out);
  write_dword<<<grid, block>>>(b, n);
  read_soa<<<(n_envs + 255) / 256, 256>>>(a, nf, n_envs, out);
  CHECK(hipDeviceSynchronize());
  printf("{\"read_bytes\": %zu, \"write_bytes\": %zu, \"out_bytes_dword\": %zu, "
         "\"out_bytes_soa\": %zu}\n", n * 4, n * 4, (size_t)grid * block * 4, (size_t)n_envs * 4);
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  CHECK(hipFree(out));
  return 0;
}
