// Host-side check of the descriptor kernel's tile cut (bcp_internal.h):
// count_tiles (O(nsrc), used by the engine to size the batch) must equal the
// per-subtile rule desc_tiles applies on the device (tile_starts over
// sub_class), and the device's tiles (start + group extension) must cover
// every subtile exactly once.  Built with hipcc, runs on the CPU.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#include "bcp_internal.h"

using namespace bcp;

int main() {
  std::mt19937_64 rng(12345);
  long checked = 0, bad = 0;
  for (int it = 0; it < 60000; it++) {
    const uint64_t T = 4096ull << (rng() % 5);  // U = 1, 2, 4, 8, 16
    const uint32_t nsrc = (uint32_t)(rng() % 13);
    std::vector<uint64_t> lens(nsrc);
    const int mode = (int)(rng() % 4);
    for (auto &L : lens) {
      switch (mode) {
        case 0: L = rng() % (20 * T); break;                                   // anywhere
        case 1: L = (rng() % 20) * T; break;                                   // subtile aligned
        case 2: L = (rng() % 20) * T + (rng() % 3 == 0 ? rng() % 32 : 0); break;  // near boundaries
        default: L = (rng() % 3) * T * 7 + rng() % (2 * T); break;
      }
    }
    std::sort(lens.begin(), lens.end(), [](uint64_t a, uint64_t b) { return a > b; });
    const uint64_t mx = nsrc ? lens[0] : 0;
    const uint64_t out_len = (rng() % 5 == 0) ? mx / 2 : mx;  // rebuild truncation too
    auto len_at = [&](uint32_t k) { return lens[k]; };
    const uint64_t nsub = (out_len + T - 1) / T;
    // device rule: one start per tile, groups extended while no new start
    uint64_t starts = 0, covered = 0;
    SubClass prev{0, 0, false};
    for (uint64_t i = 0; i < nsub; i++) {
      const SubClass cur = sub_class(len_at, nsrc, out_len, T, i);
      const SubClass pv = i ? sub_class(len_at, nsrc, out_len, T, i - 1) : SubClass{0, 0, false};
      if (pv.nf != prev.nf || pv.na != prev.na || pv.g != prev.g) bad++;
      if (tile_starts(pv, cur, i, T)) {
        starts++;
        uint64_t m = 1;
        if (cur.g) {
          const uint64_t mmax = (uint64_t)group_rows((int)(T / 4096)) / cur.nf;
          while (m < mmax && i + m < nsub &&
                 !tile_starts(cur, sub_class(len_at, nsrc, out_len, T, i + m), i + m, T))
            m++;
        }
        covered += m;
      }
      prev = cur;
    }
    const uint64_t fast = count_tiles(len_at, nsrc, out_len, T, false);
    checked++;
    if (fast != starts || covered != nsub) {
      bad++;
      if (bad < 10) {
        fprintf(stderr, "mismatch: T=%llu out_len=%llu fast=%llu starts=%llu covered=%llu nsub=%llu lens:",
                (unsigned long long)T, (unsigned long long)out_len, (unsigned long long)fast,
                (unsigned long long)starts, (unsigned long long)covered, (unsigned long long)nsub);
        for (auto L : lens) fprintf(stderr, " %llu", (unsigned long long)L);
        fprintf(stderr, "\n");
      }
    }
    if (count_tiles(len_at, nsrc, out_len, T, true) != nsub) bad++;
  }
  printf("checked %ld stripes, %ld mismatches\n", checked, bad);
  return bad ? 1 : 0;
}
