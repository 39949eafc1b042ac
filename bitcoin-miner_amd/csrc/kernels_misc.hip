// kernels_misc.hip -- k_scan instances of the classic straddling layout (C2 = 1, J = 1),
// the two-word uniform loop (C2 = 2) and the extra-padding-block layouts (EX, J = 13..15).
// Built with -mllvm -amdgpu-sched-strategy=max-ilp (Makefile): classic +2.6%, EX +0.7%,
// C2 = 2 -0.2% vs defaults; 8 waves/SIMD costs EX 3% (profiles/r01_variants.jsonl).
#include "scan_decl.h"
#include "scan_kernel.h"

GPUHASH_INSTANTIATE_SCAN(1, 1, false, 0);
GPUHASH_INSTANTIATE_SCAN(1, 1, false, 1);
GPUHASH_INSTANTIATE_SCAN(1, 2, false, 0);
GPUHASH_INSTANTIATE_SCAN(1, 2, false, 1);
GPUHASH_INSTANTIATE_SCAN(13, 0, true, 0);
GPUHASH_INSTANTIATE_SCAN(13, 0, true, 1);
GPUHASH_INSTANTIATE_SCAN(14, 0, true, 0);
GPUHASH_INSTANTIATE_SCAN(14, 0, true, 1);
GPUHASH_INSTANTIATE_SCAN(15, 0, true, 0);
GPUHASH_INSTANTIATE_SCAN(15, 0, true, 1);
