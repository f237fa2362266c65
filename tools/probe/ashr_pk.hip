// Probe (GPU box, tools only): the bit layout of gfx950's v_ashr_pk_u8_i32 (and its op_sel:[0,0,0,1] form),
// which the decoder uses to saturate and pack clipped samples. Prints D for a grid of inputs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const int32_t* a, const int32_t* b, const uint32_t* s, uint32_t* d, uint32_t* e, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t r, q;
    uint32_t init = 0xA5A5A5A5u, init2 = 0x5A5A5A5Au;
    r = init;
    q = init2;
    asm volatile("v_ashr_pk_u8_i32 %0, %1, %2, %3" : "+v"(r) : "v"(a[i]), "v"(b[i]), "v"(s[i]));
    asm volatile("v_ashr_pk_u8_i32 %0, %1, %2, %3 op_sel:[0,0,0,1]" : "+v"(q) : "v"(a[i]), "v"(b[i]), "v"(s[i]));
    d[i] = r;
    e[i] = q;
}
int main() {
    const int32_t A[] = {0, 255, 256, 65535, 65536, -1, -256, 300 << 7, 12 << 7, 0x7fffffff, -100000, 77 << 14, (-5) << 14, 1 << 20};
    const int32_t B[] = {1, 254, 511, 128, -7, 99 << 8, 300 << 8, 5 << 7, 250 << 7, 3, 255 << 14, 4, 9 << 14, -1};
    const uint32_t S[] = {0, 0, 1, 8, 8, 8, 8, 7, 7, 31, 14, 14, 14, 36};
    const int n = sizeof(A) / sizeof(A[0]);
    int32_t *da, *db; uint32_t *ds, *dd, *de;
    hipMalloc(&da, 4 * n); hipMalloc(&db, 4 * n); hipMalloc(&ds, 4 * n); hipMalloc(&dd, 4 * n); hipMalloc(&de, 4 * n);
    hipMemcpy(da, A, 4 * n, hipMemcpyHostToDevice);
    hipMemcpy(db, B, 4 * n, hipMemcpyHostToDevice);
    hipMemcpy(ds, S, 4 * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, ds, dd, de, n);
    uint32_t D[64], E[64];
    hipMemcpy(D, dd, 4 * n, hipMemcpyDeviceToHost);
    hipMemcpy(E, de, 4 * n, hipMemcpyDeviceToHost);
    for (int i = 0; i < n; ++i)
        printf("a=%d b=%d s=%u  u8: %08x  u8 op_sel hi: %08x\n", A[i], B[i], S[i], D[i], E[i]);
    return 0;
}
