// pbs1024_plan.hpp — how a batched N = 1024, k = 1, l = 3 PBS call (cfg2) is split over the
// kernels of pbs.hip and pbs1024_hex.hip (round 6).
//
// Both kernels run one workgroup per CU (LDS-bound), so a launch proceeds in rounds of
// (ciphertexts per workgroup) x CUs and a partial round costs a whole one:
//   pair kernel, 4 per CU:   a round of 4 x CUs ciphertexts in ~10.20 ms (pbs1024_pair_kernel<4>)
//   six-wave kernel, 2 per CU: a round of 2 x CUs in ~5.45 ms (pbs1024_hex_kernel<2>)
//   six-wave kernel, 1 per CU: a round of CUs in ~4.85 ms (pbs1024_hex_kernel<1>)
// (cfg2 at n = 630 on one MI355X: profiles/r05/ab5_sweep.json and profiles/r06/batch_sweep.json;
// the ratios, not the absolute times, decide the plan, and they hold for any n since every kernel's
// time is linear in n.)  Round 5 ran a whole call on ONE kernel, so a batch between round sizes
// paid a partial round of the slower choice: B = 768 ran at 75k PBS/s against 100k at 1024.  The
// call is now cut into contiguous parts, one per kernel, launched back to back on the caller's
// stream: whole pair rounds, then six-wave rounds, then at most one single-ciphertext round —
// the split of minimum estimated time.  The reference sizes its GPU chunks to the device the same
// way, in whole batches per device (compiler lib/Runtime/GPUDFG.cpp:687-731).
#pragma once
#include <stdint.h>

namespace chip {

// round costs (1/100 ms at n = 630); only their ratios matter
constexpr uint32_t PLAN_COST_PAIR = 1020, PLAN_COST_HEX2 = 545, PLAN_COST_HEX1 = 485;

struct Pbs1024Plan {
  uint32_t pair, hex2, hex1;  // ciphertexts of each part, in launch order (pair, hex2, hex1)
  uint64_t cost;              // estimated time, PLAN_COST units
};

// time of r ciphertexts on the six-wave kernel alone: whole rounds of 2 x CUs, a last partial round
// of <= CUs on one ciphertext per workgroup
inline Pbs1024Plan plan_hex_only(uint64_t r, uint64_t cus) {
  const uint64_t full = r / (2 * cus), rest = r - full * 2 * cus;
  Pbs1024Plan p{0, 0, 0, 0};
  if (rest == 0) {
    p.hex2 = (uint32_t)r;
    p.cost = full * PLAN_COST_HEX2;
  } else if (rest <= cus) {
    p.hex2 = (uint32_t)(r - rest);
    p.hex1 = (uint32_t)rest;
    p.cost = full * PLAN_COST_HEX2 + PLAN_COST_HEX1;
  } else {
    p.hex2 = (uint32_t)r;
    p.cost = (full + 1) * PLAN_COST_HEX2;
  }
  return p;
}

// the cheapest split of B ciphertexts: a whole pair rounds (the last one possibly partial, when the
// pair kernel takes everything) and the rest on the six-wave kernel
inline Pbs1024Plan plan_pbs1024(uint64_t B, uint64_t cus) {
  if (cus == 0) cus = 1;
  const uint64_t pr = 4 * cus;
  Pbs1024Plan best = plan_hex_only(B, cus);
  for (uint64_t a = 1; a <= (B + pr - 1) / pr; ++a) {
    Pbs1024Plan p;
    if (a * pr >= B) {
      p = Pbs1024Plan{(uint32_t)B, 0, 0, a * PLAN_COST_PAIR};
    } else {
      p = plan_hex_only(B - a * pr, cus);
      p.pair = (uint32_t)(a * pr);
      p.cost += a * PLAN_COST_PAIR;
    }
    if (p.cost < best.cost) best = p;
  }
  return best;
}

}  // namespace chip
