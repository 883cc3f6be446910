// msincos (wasm-pathtracer_amd/csrc/wpt_math.h) against msin / mcos, bit for
// bit, over every float of [0, 9pi/4] (argv[1]: step), its precondition.
// Build: g++ -O2 -ffp-contract=off -I wasm-pathtracer_amd/csrc tools/sincos_check.cpp
#include "wpt_math.h"
#include <cstdlib>
#include <cstdio>
#include <cstring>
using namespace wpt;
int main(int argc, char** argv) {
  uint32_t step = argc > 1 ? atoi(argv[1]) : 1;
  uint64_t bad = 0, n = 0;
  for (uint64_t u = 0; u <= 0x40e231d5u + (uint64_t)step; u += step) {
    if (u > 0x40e231d5u) u = 0x40e231d5u;  // the range's last float, whatever the step
    float x = u2f((uint32_t)u), s, c;
    msincos(x, s, c);
    float s0 = msin(x), c0 = mcos(x);
    if (f2u(s) != f2u(s0) || f2u(c) != f2u(c0)) { if (bad < 5) printf("bad %08x\n", (unsigned)u); bad++; }
    n++;
    if (u == 0x40e231d5u) break;
  }
  printf("checked %llu, mismatches %llu\n", (unsigned long long)n, (unsigned long long)bad);
  return bad != 0;
}
