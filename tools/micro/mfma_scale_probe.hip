// Probe of v_mfma_scale_f32_16x16x128_f8f6f4's scale operands (gfx950): one
// wave, one MFMA on caller-provided operand words and scale dwords, so the
// host can find which lane / byte of a scale VGPR scales which (row, K-block)
// of each operand (tools/mfma_scale_probe.py). Built by the same script:
//   hipcc --offload-arch=gfx950 -O2 -shared -fPIC tools/micro/mfma_scale_probe.hip -o tools/micro/mfma_scale_probe.so
#include <hip/hip_runtime.h>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

template <int OA, int OB>
__global__ void probe(const int* a, const int* b, const int* sa, const int* sb, float* out) {
  const int l = threadIdx.x;
  v8i A, B;
  for (int i = 0; i < 8; ++i) {
    A[i] = a[l * 8 + i];
    B[i] = b[l * 8 + i];
  }
  v4f c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A, B, c, 0, 0, OA, sa[l], OB, sb[l]);
  for (int i = 0; i < 4; ++i) out[l * 4 + i] = c[i];
}

#define CASE(x, y) \
  case x * 4 + y: hipLaunchKernelGGL((probe<x, y>), dim3(1), dim3(64), 0, 0, a, b, sa, sb, out); break;
extern "C" int probe_run(int oa, int ob, const int* a, const int* b, const int* sa, const int* sb, float* out) {
  switch (oa * 4 + ob) {
    CASE(0, 0) CASE(0, 1) CASE(0, 2) CASE(0, 3) CASE(1, 0) CASE(1, 1) CASE(1, 2) CASE(1, 3)
    CASE(2, 0) CASE(2, 1) CASE(2, 2) CASE(2, 3) CASE(3, 0) CASE(3, 1) CASE(3, 2) CASE(3, 3)
    default: return -1;
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
