// Checks the DPP wave helpers of zig-bpe_amd/csrc/wave.hpp against their definitions on random data:
// wave_shr1 / wave_shl1 (lane i <- lane i -/+ 1, the edge lane <- fill), lane_bcast, wave_incl_scan_dpp.
//   hipcc -O3 --offload-arch=gfx950 -o tools/dpp_check tools/dpp_check.hip && tools/dpp_check
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../zig-bpe_amd/csrc/wave.hpp"

using namespace zbpe;

constexpr int WAVES = 64;

__global__ void dpp_kernel(const uint32_t *in, uint32_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t x = in[i], fill = in[i ^ 63] | 1u;  // (a per-wave value: lane 0's partner)
    const uint32_t f = lane_bcast(fill, 0);
    uint32_t *o = out + (size_t)i * 5;
    o[0] = wave_shr1(x, f);
    o[1] = wave_shl1(x, f);
    o[2] = lane_bcast(x, 63);
    o[3] = wave_incl_scan_dpp(x & 0xFFFF);
    o[4] = f;
}

int main() {
    const int n = WAVES * 64;
    uint32_t *h_in = (uint32_t *)malloc(n * 4), *h_out = (uint32_t *)malloc(n * 20);
    srand(12345);
    for (int i = 0; i < n; i++) h_in[i] = ((uint32_t)rand() << 16) ^ (uint32_t)rand();
    uint32_t *d_in, *d_out;
    if (hipMalloc(&d_in, n * 4) != hipSuccess || hipMalloc(&d_out, n * 20) != hipSuccess) return 2;
    (void)hipMemcpy(d_in, h_in, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(dpp_kernel, dim3(WAVES / 4), dim3(256), 0, 0, d_in, d_out);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    (void)hipMemcpy(h_out, d_out, n * 20, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int w = 0; w < WAVES; w++) {
        uint32_t sum = 0;
        for (int l = 0; l < 64; l++) {
            const int i = w * 64 + l;
            const uint32_t *o = h_out + (size_t)i * 5, f = o[4];
            sum += h_in[i] & 0xFFFF;
            const uint32_t e[4] = {l ? h_in[i - 1] : f, l < 63 ? h_in[i + 1] : f, h_in[w * 64 + 63], sum};
            for (int k = 0; k < 4; k++)
                if (o[k] != e[k] && bad++ < 8) printf("wave %d lane %d op %d: got %08x want %08x\n", w, l, k, o[k], e[k]);
        }
    }
    printf("{\"dpp_check\": \"%s\", \"mismatches\": %d, \"lanes\": %d}\n", bad ? "FAIL" : "ok", bad, n);
    return bad ? 1 : 0;
}
