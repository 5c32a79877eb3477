// VALU issue-rate probe (gfx950): how many cycles of SIMD throughput does a
// wave64 integer VALU instruction of the codelets' kind (v_sub_u32_sdwa fold,
// v_mul_i32_i24, v_add_u32) cost at 1, 2, 4, 8 waves per SIMD?
//   hipcc --offload-arch=gfx950 -O3 -o build/valu_probe tools/valu_probe.hip
// Each lane runs CH independent chains of ITER x (mul_i24, fold, add); the
// number of resident waves per SIMD is set by dynamic LDS (one 256-thread
// block per CU per 40 KB...).  Prints cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-result"

#include <cstdio>
#include <vector>

constexpr int CH = 8, ITER = 4096;

__global__ __launch_bounds__(256) void probe(int* out, int c, unsigned long long* clk)
{
    extern __shared__ int lds[];
    int v[CH];
#pragma unroll
    for (int i = 0; i < CH; i++)
        v[i] = threadIdx.x + i * 7;
    int cb;
    asm volatile("s_mov_b32 %0, %1" : "=s"(cb) : "s"(c));
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int i = 0; i < CH; i++) {
            int x, y;
            asm("v_mul_i32_i24 %0, %1, %2" : "=v"(x) : "s"(cb), "v"(v[i]));
            asm("v_sub_u32_sdwa %0, %1, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD "
                "src0_sel:WORD_0 src1_sel:WORD_1"
                : "=v"(y)
                : "v"(x));
            asm("v_add_u32 %0, %1, %2" : "=v"(v[i]) : "v"(y), "v"(cb));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int s = 0;
#pragma unroll
    for (int i = 0; i < CH; i++)
        s += v[i];
    if (s == 0x7fffffff)
        lds[0] = s;  // keep the LDS allocation
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0)
        clk[blockIdx.x] = t1 - t0;
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int* out;
    unsigned long long* clk;
    hipMalloc(&out, 256 * 8 * cus * sizeof(int));
    hipMalloc(&clk, 8 * cus * sizeof(unsigned long long));
    // blocks per CU b -> waves per SIMD = b (256 threads = 4 waves, one per SIMD)
    for (int b : {1, 2, 3, 4, 6, 8}) {
        const size_t lds = 160 * 1024 / b - 1024;
        hipFuncSetAttribute(reinterpret_cast<const void*>(&probe),
                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
        const int grid = cus * b;
        hipLaunchKernelGGL(probe, dim3(grid), dim3(256), lds, 0, out, 12345, clk);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        for (int r = 0; r < 5; r++)
            hipLaunchKernelGGL(probe, dim3(grid), dim3(256), lds, 0, out, 12345, clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<unsigned long long> c(grid);
        hipMemcpy(c.data(), clk, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        double avg = 0;
        for (auto x : c)
            avg += static_cast<double>(x);
        avg /= grid;
        // VALU instructions per wave in the loop: 3 per chain step
        const double instr = 3.0 * CH * ITER;
        // s_memtime counts shader cycles; per wave: avg cycles / instr is the
        // wave's own issue interval; b waves share a SIMD
        printf("waves/SIMD %d: %.2f cycles per wave-instr (wave view), %.2f cycles per "
               "instr per SIMD; wall %.3f ms/launch, clock %.2f GHz\n",
               b, avg / instr, avg / instr / b, ms / 5,
               avg / (ms / 5 * 1e-3) / 1e9);
    }
    return 0;
}
