// Diagnostic (not part of the library): HBM write rate of 16-byte-per-lane vector stores by how the 64
// lanes of one store instruction map onto rows of 1 KiB (the point-form row stores of the chains and
// projections write 16 rows x 64 B per instruction).
//   hipcc --offload-arch=gfx950 -O3 store_shape.hip -o store_shape && ./store_shape
#include <hip/hip_runtime.h>
#include <cstdio>

// rows of 256 floats (1 KiB); shape R = rows per instruction (64 lanes x 16 B = 1 KiB = R rows x (1024/R) B)
template <int R>
__global__ void __launch_bounds__(256) store_rows(float4* __restrict__ y, long nrows) {
  constexpr int SEG = 64 / R;                 // lanes (16 B each) per row segment
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long rows_per_wave = 16;              // every wave owns 16 consecutive rows (the point form)
  const long r0 = ((long)blockIdx.x * 4 + wave) * rows_per_wave;
  if (r0 >= nrows) return;
  const float4 v = make_float4(1.f, 2.f, 3.f, (float)lane);
  // 16 rows x 64 float4: 16 instructions; instruction i covers rows r0 + (i*R ... ) in R-row bands
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    // R = 16: lane -> row lane & 15, column segment 4 * (lane >> 4) + 16 * i  (the point form)
    // R = 4: lane -> row 4 * (i & 3) + (lane >> 4), float4 column (lane & 15) + 16 * (i >> 2)
    // R = 1: lane -> row i, float4 column lane (and a second 64-lane half of the row is another instr)
    long row; int col4;
    if (R == 16) { row = r0 + (lane & 15); col4 = 4 * i + (lane >> 4); }
    else if (R == 4) { row = r0 + 4 * (i & 3) + (lane >> 4); col4 = (lane & 15) + 16 * (i >> 2); }
    else { row = r0 + i; col4 = lane; }
    y[row * 64 + col4] = v;
  }
}

template <int R>
static float run(float4* y, long nrows) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  const int blocks = (int)((nrows / 16 + 3) / 4);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(store_rows<R>, dim3(blocks), dim3(256), 0, 0, y, nrows);
  (void)hipEventRecord(a, 0);
  for (int w = 0; w < 10; ++w) hipLaunchKernelGGL(store_rows<R>, dim3(blocks), dim3(256), 0, 0, y, nrows);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  const long nrows = 1L << 20;                // 1 GiB of 1 KiB rows
  float4* y;
  if (hipMalloc(&y, nrows * 1024) != hipSuccess) return 1;
  // R = 16 covers 16 rows x 64 B per instruction but only 16 float4 of each row per pass of i: 16 instrs
  // write 16 rows x 1 KiB; R = 1: 16 instrs write 16 rows x 1 KiB (each instr one row's first/second half?)
  float t16 = run<16>(y, nrows), t4 = run<4>(y, nrows), t1 = run<1>(y, nrows);
  printf("16 rows x 64 B per instruction : %.3f ms  %.2f TB/s\n", t16, nrows * 1024 / t16 / 1e9);
  printf(" 4 rows x 256 B per instruction: %.3f ms  %.2f TB/s\n", t4, nrows * 1024 / t4 / 1e9);
  printf(" 1 row  x 1 KiB per instruction: %.3f ms  %.2f TB/s\n", t1, nrows * 1024 / t1 / 1e9);
  (void)hipFree(y);
  return 0;
}
