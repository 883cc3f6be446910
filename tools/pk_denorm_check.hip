// Checks on the GPU that packed f32 subtract / multiply (v_pk_add_f32 /
// v_pk_mul_f32, what expand_pair's slab terms compile to) give the same bits
// as the scalar IEEE ops, denormal inputs and results included.
// Build: hipcc -O3 -ffp-contract=off -fno-gpu-flush-denormals-to-zero --offload-arch=gfx950 -o tools/pk_denorm_check tools/pk_denorm_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
typedef float f2v __attribute__((ext_vector_type(2)));
__global__ void k(const float* a, const float* o, const float* inv, uint32_t n, uint32_t* bad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  const float a0 = a[2 * i], a1 = a[2 * i + 1], oo = o[i], ii = inv[i];
  const float s0 = (a0 - oo) * ii, s1 = (a1 - oo) * ii;
  const f2v av = {a0, a1}, ov = {oo, oo}, iv = {ii, ii};
  const f2v p = (av - ov) * iv;
  if (__float_as_uint(p.x) != __float_as_uint(s0) || __float_as_uint(p.y) != __float_as_uint(s1)) atomicAdd(bad, 1u);
}
static uint32_t xs = 2463534242u;
static uint32_t rnd() { xs ^= xs << 13; xs ^= xs >> 17; xs ^= xs << 5; return xs; }
static float pick() {
  uint32_t r = rnd(), m = r % 4;
  float f;
  uint32_t u = rnd();
  if (m == 0) u &= 0x807FFFFFu;                          // denormal (or zero)
  else if (m == 1) u = (u & 0x80FFFFFFu) | 0x00800000u;  // smallest normal binade
  memcpy(&f, &u, 4);
  if (m == 3) f = (float)((int)(r % 2001) - 1000) * 0.37f;
  return f;
}
int main() {
  const uint32_t n = 1u << 24;
  std::vector<float> a(n), o(n / 2), inv(n / 2);
  for (auto& x : a) x = pick();
  for (uint32_t i = 0; i < n / 2; i++) {
    o[i] = (i & 1) ? a[2 * i] * 0.999f : pick();  // close operands: denormal differences
    inv[i] = (i & 2) ? 1.0f / pick() : pick();
  }
  float *da, *dob, *di;
  uint32_t* db;
  hipMalloc(&da, n * 4); hipMalloc(&dob, n * 2); hipMalloc(&di, n * 2); hipMalloc(&db, 4);
  hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(dob, o.data(), n * 2, hipMemcpyHostToDevice);
  hipMemcpy(di, inv.data(), n * 2, hipMemcpyHostToDevice);
  hipMemset(db, 0, 4);
  k<<<n / 2 / 256, 256>>>(da, dob, di, n, db);
  uint32_t bad = 0;
  hipMemcpy(&bad, db, 4, hipMemcpyDeviceToHost);
  printf("{\"pairs\": %u, \"mismatches\": %u}\n", n / 2, bad);
  return bad != 0;
}
