// Checks the DPP wave helpers of zig-bpe_amd/csrc/wave.hpp against their definitions on random data:
// wave_shr1 / wave_shl1 (lane i <- lane i -/+ 1, the edge lane <- fill), lane_bcast, wave_incl_scan_dpp,
// wave_max_u32, wave_sum_u32, and kernels.hpp's DPP reductions: the ordered carry-summary scan (summ_scan_dpp,
// summ_excl_dpp, wave_reduce_summ), the argmax's wave_max_dpp, the tie decision's wave_minK_reduce_dpp and the
// self-pair run-parity block scan (self_block_scan, a 256-thread block).
//   hipcc -O3 --offload-arch=gfx950 -o tools/dpp_check tools/dpp_check.hip && tools/dpp_check
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../zig-bpe_amd/csrc/kernels.hpp"

using namespace zbpe;

constexpr int WAVES = 64;
constexpr int NOUT = 23;

__global__ void dpp_kernel(const uint32_t *in, uint32_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t x = in[i], fill = in[i ^ 63] | 1u;  // (a per-wave value: lane 0's partner)
    const uint32_t f = lane_bcast(fill, 0);
    uint32_t *o = out + (size_t)i * NOUT;
    o[0] = wave_shr1(x, f);
    o[1] = wave_shl1(x, f);
    o[2] = lane_bcast(x, 63);
    o[3] = wave_incl_scan_dpp(x & 0xFFFF);
    o[4] = f;
    o[5] = wave_max_u32(x);
    o[6] = wave_sum_u32(x & 0xFFFF);
    // a carry summary per lane (one home slot's count 0..3: m >= max(q, 0) as every summary has)
    const Summ sx = summ_slot(x & 3u);
    const Summ inc = summ_scan_dpp(sx), ex = summ_excl_dpp(inc), red = wave_reduce_summ(sx);
    o[7] = (uint32_t)inc.q; o[8] = (uint32_t)inc.m; o[9] = (uint32_t)ex.q; o[10] = (uint32_t)ex.m;
    o[11] = (uint32_t)red.q; o[12] = (uint32_t)red.m;
    // argmax records: counts in 0..7 (ties), ids = the lane
    const MaxRec mr = wave_max_dpp(MaxRec{x & 7u, (x & 7u) ? 1u : 0u, (x & 7u) ? (threadIdx.x & 63u) : NO_ID});
    o[13] = mr.cnt | (mr.ties << 8) | (mr.id << 16);
    // the three smallest distinct 64-bit entries (home << 32 | lane) and the largest home
    uint64_t q[3] = {((uint64_t)(x >> 8) << 32) | (threadIdx.x & 63u), ~0ull, ~0ull};
    uint32_t hm = x >> 8;
    wave_minK_reduce_dpp<3>(q, hm);
    for (int k = 0; k < 3; k++) { o[14 + 2 * k] = (uint32_t)q[k]; o[15 + 2 * k] = (uint32_t)(q[k] >> 32); }
    o[20] = hm;
    __shared__ uint8_t s_wave[SELF_THREADS / 64];
    uint8_t tot = 0;
    o[21] = self_block_scan((uint8_t)(x & 3u), s_wave, &tot);
    o[22] = tot;
}

// host restatement of self_compose (g after f)
static uint8_t self_compose_h(uint8_t f, uint8_t g) { return (g & 1) ? (uint8_t)((f & 1) | ((f ^ g) & 2)) : g; }

int main() {
    const int n = WAVES * 64;
    uint32_t *h_in = (uint32_t *)malloc(n * 4), *h_out = (uint32_t *)malloc((size_t)n * NOUT * 4);
    srand(12345);
    for (int i = 0; i < n; i++) h_in[i] = ((uint32_t)rand() << 16) ^ (uint32_t)rand();
    uint32_t *d_in, *d_out;
    if (hipMalloc(&d_in, n * 4) != hipSuccess || hipMalloc(&d_out, (size_t)n * NOUT * 4) != hipSuccess) return 2;
    (void)hipMemcpy(d_in, h_in, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(dpp_kernel, dim3(WAVES / 4), dim3(256), 0, 0, d_in, d_out);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    (void)hipMemcpy(h_out, d_out, (size_t)n * NOUT * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int w = 0; w < WAVES; w++) {
        uint32_t sum = 0, wmax = 0, wsum = 0, mc = 0, mt = 0, mi = 0xFFFF;
        int32_t tq = 0, tm = 0;  // the wave's ordered composition
        for (int l = 0; l < 64; l++) {
            const uint32_t v = h_in[w * 64 + l];
            wmax = v > wmax ? v : wmax;
            wsum += v & 0xFFFF;
            const int32_t q = (int32_t)(v & 3u) - 1, m = q > 0 ? q : 0;
            tm = m > tm + q ? m : tm + q;
            tq += q;
            const uint32_t c = v & 7u;
            if (c > mc) { mc = c; mt = 1; mi = (uint32_t)l; } else if (c && c == mc) mt++;
        }
        const uint32_t mrec = mc | (mt << 8) | ((mc ? mi : 0xFFFFu) << 16);
        uint64_t k3[3] = {~0ull, ~0ull, ~0ull};
        uint32_t hm = 0;
        for (int l = 0; l < 64; l++) {
            const uint64_t e = ((uint64_t)(h_in[w * 64 + l] >> 8) << 32) | (uint32_t)l;
            hm = (h_in[w * 64 + l] >> 8) > hm ? (h_in[w * 64 + l] >> 8) : hm;
            if (e < k3[0]) { k3[2] = k3[1]; k3[1] = k3[0]; k3[0] = e; }
            else if (e < k3[1]) { k3[2] = k3[1]; k3[1] = e; }
            else if (e < k3[2]) k3[2] = e;
        }
        int32_t pq = 0, pm = 0;  // the running inclusive composition
        // the run-parity functions (bit0: all a, bit1: parity) composed over the block (4 waves) before each thread
        const int blk0 = (w / 4) * 256;
        uint8_t bt = 1;
        for (int t = 0; t < 256; t++) bt = self_compose_h(bt, (uint8_t)(h_in[blk0 + t] & 3u));
        uint8_t run = 1;
        for (int t = blk0; t < w * 64; t++) run = self_compose_h(run, (uint8_t)(h_in[t] & 3u));
        for (int l = 0; l < 64; l++) {
            const int i = w * 64 + l;
            const uint32_t *o = h_out + (size_t)i * NOUT, f = o[4];
            sum += h_in[i] & 0xFFFF;
            const int32_t eq = pq, em = pm;  // the exclusive composition
            {
                const int32_t q = (int32_t)(h_in[i] & 3u) - 1, m = q > 0 ? q : 0;
                pm = m > pm + q ? m : pm + q;
                pq += q;
            }
            const uint8_t ex_self = run;
            run = self_compose_h(run, (uint8_t)(h_in[i] & 3u));
            const uint32_t e[23] = {l ? h_in[i - 1] : f, l < 63 ? h_in[i + 1] : f, h_in[w * 64 + 63], sum, f, wmax, wsum,
                                    (uint32_t)pq, (uint32_t)pm, (uint32_t)eq, (uint32_t)em, (uint32_t)tq, (uint32_t)tm, mrec,
                                    (uint32_t)k3[0], (uint32_t)(k3[0] >> 32), (uint32_t)k3[1], (uint32_t)(k3[1] >> 32),
                                    (uint32_t)k3[2], (uint32_t)(k3[2] >> 32), hm, ex_self, bt};
            for (int k = 0; k < 23; k++)
                if (o[k] != e[k] && bad++ < 8) printf("wave %d lane %d op %d: got %08x want %08x\n", w, l, k, o[k], e[k]);
        }
    }
    printf("{\"dpp_check\": \"%s\", \"mismatches\": %d, \"lanes\": %d}\n", bad ? "FAIL" : "ok", bad, n);
    return bad ? 1 : 0;
}
