// kernels_plain.hip -- k_scan instances of the plain layouts (C2 = 0, no extra block):
// loop word W_J of the only nonce-bearing block, J = 0..13.  Built with
// -DGPUHASH_WAVES_PER_EU=8 (Makefile): 8 waves/SIMD in 63 VGPRs without spills, +0.3% on
// config 2 and +4% on J = 2 over the unconstrained build (profiles/r01_variants.jsonl).
#include "scan_decl.h"
#include "scan_kernel.h"

#define PLAIN(J) GPUHASH_INSTANTIATE_SCAN(J, 0, false, 0); GPUHASH_INSTANTIATE_SCAN(J, 0, false, 1)
PLAIN(0);
PLAIN(1);
PLAIN(2);
PLAIN(3);
PLAIN(4);
PLAIN(5);
PLAIN(6);
PLAIN(7);
PLAIN(8);
PLAIN(9);
PLAIN(10);
PLAIN(11);
PLAIN(12);
PLAIN(13);
