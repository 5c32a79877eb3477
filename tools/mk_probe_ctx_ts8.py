#!/usr/bin/env python3
"""Writes the stage-stamp probe of the k <= 128 context kernel
(tools/ctx_stages8.py) into a copy of ctx.hip:
    python3 tools/mk_probe_ctx_ts8.py <ctx.hip in> <ctx.hip out>"""
import sys

s = open(sys.argv[1]).read()


def rep(old, new):
    global s
    assert s.count(old) == 1, old
    s = s.replace(old, new)


rep("""template <int NT>
__global__ __launch_bounds__(NT) void decode_ctx_lds_kernel(""", """// PROBE: per-block stage timestamps (s_memrealtime, 100 MHz)
__device__ unsigned long long qi_ts[8192 * 8];
#define QI_TS(i) do { if (threadIdx.x == 0 && blockIdx.x < 8192) qi_ts[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
template <int NT>
__global__ __launch_bounds__(NT) void decode_ctx_lds_kernel(""")
rep("""    int32_t* mat = ctx + s * ctx_stride;
    const int kp = ctx_pitch(k);
    uint32_t* Mt = qi_ctx_lds;""", """    int32_t* mat = ctx + s * ctx_stride;
    QI_TS(0);
    const int kp = ctx_pitch(k);
    uint32_t* Mt = qi_ctx_lds;""")
rep("""    // x_i = r^{id_i}: thread tid takes point tid (its Q chain below); wave 0
    // also point 64 + lane""", """    QI_TS(1);
    // x_i = r^{id_i}: thread tid takes point tid (its Q chain below); wave 0
    // also point 64 + lane""")
rep("""    int32_t ab0 = 0;  // wave 0: balanced A[lane] (k <= 64), for the Q chains
    if (tid < 64) {""", """    int32_t ab0 = 0;  // wave 0: balanced A[lane] (k <= 64), for the Q chains
    QI_TS(2);
    if (tid < 64) {""")
rep("""        if (tid == 0)
            A[k] = 1;
    } else if (in_oor.counts) {""", """        if (tid == 0)
            A[k] = 1;
        QI_TS(3);
    } else if (in_oor.counts) {""")
rep("""    __syncthreads();
    if (tid < k) {
        // Q_i = A / (x - x_i) by synthetic division from the top, and""", """    __syncthreads();
    QI_TS(4);
    if (tid < k) {
        // Q_i = A / (x - x_i) by synthetic division from the top, and""")
rep("""    __syncthreads();
    // one pass per row, 4 lanes per row (quad reductions by DPP), lane sub""", """    __syncthreads();
    QI_TS(5);
    // one pass per row, 4 lanes per row (quad reductions by DPP), lane sub""")
rep("""    if (!dot2)
        return;
    __syncthreads();  // every row final (the pass above is row-local)""", """    __syncthreads();
    QI_TS(6);
    if (!dot2)
        return;
    __syncthreads();  // every row final (the pass above is row-local)""")
rep("""}  // namespace qi
""", """}  // namespace qi

extern "C" int qi_probe_ts(unsigned long long* h, int n)
{
    return hipMemcpyFromSymbol(h, HIP_SYMBOL(qi::qi_ts), static_cast<size_t>(n) * 8 * 8) == hipSuccess ? 0 : -1;
}
""")
open(sys.argv[2], "w").write(s)
