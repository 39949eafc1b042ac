// placement_probe.hip -- where do the 4 waves of a 256-thread workgroup run?
//
// Launches a persistent-style grid shaped like the two-word uniform scan kernel
// (k_scan<1,2,false,0>: 256 threads, 17 KB of LDS, ~96 VGPRs, so 5 workgroups per CU)
// and records, per wave, the workgroup, the wave index and the HW_ID hardware register
// (SIMD, CU, shader engine) plus XCC_ID.  Output: one line per wave
//   block wave xcc se cu simd
// for tools/placement_probe.py.  Read-only hardware registers (s_getreg), vector stores.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

// s_getreg immediate: (size - 1) << 11 | offset << 6 | register id
#define HWREG(id, off, size) (((size) - 1) << 11 | (off) << 6 | (id))

__global__ __launch_bounds__(256) void probe(unsigned* out, unsigned spin) {
    __shared__ unsigned lds[17 * 1024 / 4];
    asm volatile("; reserve v0-v95 like the scan kernel (93 VGPRs)" ::: "v95");
    const unsigned tid = threadIdx.x;
    lds[tid] = tid;
    __syncthreads();
    // keep every wave resident for a while so the dispatcher fills the CU
    unsigned x = lds[(tid * 7) & 255];
    for (unsigned i = 0; i < spin; i++) x = x * 1664525u + 1013904223u;
    const unsigned hw = __builtin_amdgcn_s_getreg(HWREG(4, 0, 32));    // HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg(HWREG(20, 0, 16));  // XCC_ID
    if ((tid & 63u) == 0) {
        unsigned* o = out + 4 * (blockIdx.x * 4 + (tid >> 6));
        o[0] = hw;
        o[1] = xcc;
        o[2] = x;  // keeps the spin loop alive
        o[3] = 1;
    }
}

int main(int argc, char** argv) {
    const int per_cu = argc > 1 ? atoi(argv[1]) : 5;
    const unsigned spin = argc > 2 ? (unsigned)atoi(argv[2]) : 200000;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
    int occ = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, probe, 256, 0);
    const int grid = prop.multiProcessorCount * per_cu;
    fprintf(stderr, "CUs %d occupancy %d blocks/CU, grid %d\n", prop.multiProcessorCount, occ, grid);
    unsigned* d = nullptr;
    const size_t bytes = (size_t)grid * 4 * 4 * sizeof(unsigned);
    if (hipMalloc(&d, bytes) != hipSuccess) return 1;
    hipMemset(d, 0, bytes);
    hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, 0, d, spin);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    unsigned* h = (unsigned*)malloc(bytes);
    hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost);
    printf("occupancy %d\n", occ);
    for (int b = 0; b < grid; b++)
        for (int w = 0; w < 4; w++) {
            const unsigned* o = h + 4 * (b * 4 + w);
            const unsigned hw = o[0];
            // gfx9 HW_ID: WAVE_ID[3:0] SIMD_ID[5:4] PIPE_ID[7:6] CU_ID[11:8] SH_ID[12] SE_ID[15:13]
            printf("%d %d %u %u %u %u %u\n", b, w, o[1] & 0xF, (hw >> 13) & 7, (hw >> 8) & 15,
                   (hw >> 4) & 3, (hw >> 12) & 1);
        }
    free(h);
    hipFree(d);
    return 0;
}
