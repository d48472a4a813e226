// Probe the lane mapping of ds_read_b64_tr_b16 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4_t lds_s4;
__global__ void k(short* out, int mode) {
  __shared__ short lds[64 * 64];
  for (int i = threadIdx.x; i < 64 * 64; i += 64) lds[i] = (short)i;  // value = row*64 + col
  __syncthreads();
  int lane = threadIdx.x;
  int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  int row = 4 * g + q, col = 4 * p;           // each group reads its own 4-row block at cols 0..15
  if (mode == 1) { row = q; col = 16 * g + 4 * p; }
  short4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lds + row * 64 + col));
  for (int j = 0; j < 4; ++j) out[lane * 4 + j] = v[j];
}
int main() {
  short* d; hipMalloc(&d, 64 * 4 * 2);
  short h[256];
  for (int mode = 0; mode < 2; ++mode) {
    k<<<1, 64>>>(d, mode); hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    printf("mode %d\n", mode);
    for (int l = 0; l < 64; ++l) {
      printf("lane %2d:", l);
      for (int j = 0; j < 4; ++j) printf(" (r%2d,c%2d)", h[l * 4 + j] / 64, h[l * 4 + j] % 64);
      printf("%s", (l % 2) ? "\n" : "   ");
    }
  }
  return 0;
}
