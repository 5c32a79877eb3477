// Layout probe (not part of the product): checks, with exact integer data,
//  1. the operand / result lane maps of v_mfma_i32_16x16x32_i8,
//  2. what ds_read_b64_tr_b8 delivers per lane,
// before the matrix kernel relies on them.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_probe.hip -o build/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));

__host__ __device__ int Aval(int r, int k) { return (r * 3 + k * 5) % 11 - 5; }
__host__ __device__ int Bval(int k, int c) { return (k * 7 + c * 2) % 13 - 6; }

__global__ void mfma_test(int* out)
{
    const int l = threadIdx.x;
    // hypothesis: lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15]
    uint64_t a = 0, b = 0;
    for (int j = 0; j < 8; j++) {
        a |= (uint64_t)(uint8_t)(int8_t)Aval(l & 15, 8 * (l >> 4) + j) << (8 * j);
        b |= (uint64_t)(uint8_t)(int8_t)Bval(8 * (l >> 4) + j, l & 15) << (8 * j);
    }
    v4i c = {1000 * l, 1000 * l + 1, 1000 * l + 2, 1000 * l + 3};
    v4i d = __builtin_amdgcn_mfma_i32_16x16x32_i8((long)a, (long)b, c, 0, 0, 0);
    for (int j = 0; j < 4; j++)
        out[l * 4 + j] = d[j];
}

__global__ void tr8_test(int* out)
{
    __shared__ uint8_t img[4][128];
    const int l = threadIdx.x;
    for (int i = l; i < 512; i += 64) {
        const int g = i / 128, row = (i % 128) / 16, col = i % 16;
        img[g][row * 16 + col] = (uint8_t)(row * 16 + col);
    }
    __syncthreads();
    const int g = l >> 4, q = (l & 15) >> 1, p = l & 1;
    auto* base = (__attribute__((address_space(3))) char*)&img[0][0];
    v2i r = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
        (__attribute__((address_space(3))) v2i*)(base + g * 128 + q * 16 + 8 * p));
    out[2 * l] = r[0];
    out[2 * l + 1] = r[1];
}

int main()
{
    int *d, h[512];
    hipMalloc(&d, 4096);
    mfma_test<<<1, 64>>>(d);
    hipMemcpy(h, d, 256 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; l++)
        for (int j = 0; j < 4; j++) {
            const int row = 4 * (l >> 4) + j, col = l & 15;
            int ref = 1000 * l + j;
            for (int k = 0; k < 32; k++)
                ref += Aval(row, k) * Bval(k, col);
            if (h[l * 4 + j] != ref) {
                if (bad < 5)
                    printf("mfma mismatch lane %d reg %d got %d want %d\n", l, j,
                           h[l * 4 + j], ref);
                bad++;
            }
        }
    printf("mfma_i32_16x16x32_i8 layout hypothesis: %s (%d mismatches)\n",
           bad ? "WRONG" : "OK", bad);
    tr8_test<<<1, 64>>>(d);
    hipMemcpy(h, d, 128 * 4, hipMemcpyDeviceToHost);
    bad = 0;
    for (int l = 0; l < 64; l++) {
        const uint8_t* b = (const uint8_t*)&h[2 * l];
        for (int r = 0; r < 8; r++)
            if (b[r] != (uint8_t)(r * 16 + (l & 15)))
                bad++;
    }
    printf("ds_read_b64_tr_b8 hypothesis (lane i of a 16-lane group: column i, "
           "rows 0..7): %s (%d mismatches)\n", bad ? "WRONG" : "OK", bad);
    for (int l = 0; l < 18; l++) {
        const uint8_t* b = (const uint8_t*)&h[2 * l];
        printf("lane %2d:", l);
        for (int r = 0; r < 8; r++)
            printf(" %3d", b[r]);
        printf("\n");
    }
    return 0;
}
