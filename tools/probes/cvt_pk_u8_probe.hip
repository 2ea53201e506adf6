// Semantics probe of v_cvt_pk_u8_f32 on gfx950 (rounding mode, clamping): prints x -> byte for a
// few values.  hipcc --offload-arch=gfx950 -O2 -o /tmp/cvt_probe tools/probes/cvt_pk_u8_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(const float* x, unsigned* o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = __builtin_amdgcn_cvt_pk_u8_f32(x[i], 0, 0u);
}

int main() {
  const float xs[] = {-3.f, -0.6f, -0.5f, -0.4f, 0.f, 0.4f, 0.5f, 0.6f, 1.5f, 2.5f, 3.49f, 3.5f, 3.51f, 254.5f, 255.f, 255.4f, 255.6f, 300.f, 1e9f};
  const int n = sizeof(xs) / sizeof(xs[0]);
  float* dx;
  unsigned* dout;
  unsigned out[64];
  if (hipMalloc(&dx, sizeof(xs)) != hipSuccess || hipMalloc(&dout, n * sizeof(unsigned)) != hipSuccess) return 1;
  hipMemcpy(dx, xs, sizeof(xs), hipMemcpyHostToDevice);
  probe<<<1, 64>>>(dx, dout, n);
  hipMemcpy(out, dout, n * sizeof(unsigned), hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) printf("%g -> %u\n", xs[i], out[i] & 255u);
  hipFree(dx);
  hipFree(dout);
  return 0;
}
