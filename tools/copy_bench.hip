// Achievable HBM bandwidth probes (device-to-device copies of 4 GiB, HIP events): which copy
// shape reaches the MI355X's measured peak on this box.  Usage: ./copy_bench [GiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { if ((x) != hipSuccess) { printf("HIP error %s\n", #x); exit(1); } } while (0)

// a: grid-stride, 4 x 16 B in flight per thread (mtg_device_copy)
__global__ __launch_bounds__(256) void copy_gs4(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n) {
    const uint64_t st = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * st < n; i += 4 * st) {
        uint4 a = s[i], b = s[i + st], c = s[i + 2 * st], e = s[i + 3 * st];
        d[i] = a; d[i + st] = b; d[i + 2 * st] = c; d[i + 3 * st] = e;
    }
    for (; i < n; i += st) d[i] = s[i];
}
// b: one-shot, each thread 4 x 16 B at a block-strided offset (fully coalesced per instruction)
__global__ __launch_bounds__(256) void copy_os4(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n) {
    const uint64_t b0 = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) if (b0 + 256 * q < n) v[q] = s[b0 + 256 * q];
#pragma unroll
    for (int q = 0; q < 4; ++q) if (b0 + 256 * q < n) d[b0 + 256 * q] = v[q];
}
// c: one-shot with nontemporal loads and stores
__global__ __launch_bounds__(256) void copy_os4_nt(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n) {
    const uint64_t b0 = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (b0 + 256 * q < n) {
            const uint64_t *p = (const uint64_t *)(s + b0 + 256 * q);
            uint64_t x = __builtin_nontemporal_load(p), y = __builtin_nontemporal_load(p + 1);
            v[q] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
        }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        if (b0 + 256 * q < n) {
            uint64_t *p = (uint64_t *)(d + b0 + 256 * q);
            __builtin_nontemporal_store((uint64_t)v[q].x | (uint64_t)v[q].y << 32, p);
            __builtin_nontemporal_store((uint64_t)v[q].z | (uint64_t)v[q].w << 32, p + 1);
        }
}
// d: one-shot, 8 x 16 B per thread
__global__ __launch_bounds__(256) void copy_os8(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n) {
    const uint64_t b0 = (uint64_t)blockIdx.x * 2048 + threadIdx.x;
    uint4 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) if (b0 + 256 * q < n) v[q] = s[b0 + 256 * q];
#pragma unroll
    for (int q = 0; q < 8; ++q) if (b0 + 256 * q < n) d[b0 + 256 * q] = v[q];
}

// e: one-shot, ONE 16 B per thread (the plain float4 copy)
__global__ __launch_bounds__(256) void copy_os1(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) d[i] = s[i];
}
// f: one-shot, 2 x 16 B per thread
__global__ __launch_bounds__(256) void copy_os2(const uint4 *__restrict__ s, uint4 *__restrict__ d, uint64_t n) {
    const uint64_t b0 = (uint64_t)blockIdx.x * 512 + threadIdx.x;
    uint4 v[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) if (b0 + 256 * q < n) v[q] = s[b0 + 256 * q];
#pragma unroll
    for (int q = 0; q < 2; ++q) if (b0 + 256 * q < n) d[b0 + 256 * q] = v[q];
}
// g: one-shot 4 x 16 B with 16-byte nontemporal vector loads / stores (one instruction each)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int PER>
__global__ __launch_bounds__(256) void copy_osv_nt(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, uint64_t n) {
    const uint64_t b0 = (uint64_t)blockIdx.x * (256 * PER) + threadIdx.x;
    u32x4 v[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) if (b0 + 256 * q < n) v[q] = __builtin_nontemporal_load(s + b0 + 256 * q);
#pragma unroll
    for (int q = 0; q < PER; ++q) if (b0 + 256 * q < n) __builtin_nontemporal_store(v[q], d + b0 + 256 * q);
}
// h: one-shot 4 x 16 B, plain loads, nontemporal 16-byte stores
__global__ __launch_bounds__(256) void copy_os4_ntst(const u32x4 *__restrict__ s, u32x4 *__restrict__ d, uint64_t n) {
    const uint64_t b0 = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    u32x4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) if (b0 + 256 * q < n) v[q] = s[b0 + 256 * q];
#pragma unroll
    for (int q = 0; q < 4; ++q) if (b0 + 256 * q < n) __builtin_nontemporal_store(v[q], d + b0 + 256 * q);
}

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 4.0;
    const uint64_t bytes = (uint64_t)(gib * (1ull << 30)), n = bytes / 16;
    uint4 *s, *d;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 1, bytes));
    CK(hipMemset(d, 0, bytes));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("%-28s %.3f ms  %.2f TB/s\n", name, ms / reps, 2.0 * bytes / (ms / reps * 1e-3) / 1e12);
    };
    for (int mult : {4, 8, 16, 32})
        run(mult == 4 ? "grid-stride x4, 4 WG/CU" : mult == 8 ? "grid-stride x4, 8 WG/CU" :
            mult == 16 ? "grid-stride x4, 16 WG/CU" : "grid-stride x4, 32 WG/CU",
            [&] { copy_gs4<<<dim3(cus * mult), dim3(256)>>>(s, d, n); });
    run("one-shot 4 x 16 B", [&] { copy_os4<<<dim3((unsigned)((n + 1023) / 1024)), dim3(256)>>>(s, d, n); });
    run("one-shot 4 x 16 B nt", [&] { copy_os4_nt<<<dim3((unsigned)((n + 1023) / 1024)), dim3(256)>>>(s, d, n); });
    run("one-shot 8 x 16 B", [&] { copy_os8<<<dim3((unsigned)((n + 2047) / 2048)), dim3(256)>>>(s, d, n); });
    run("one-shot 1 x 16 B", [&] { copy_os1<<<dim3((unsigned)((n + 255) / 256)), dim3(256)>>>(s, d, n); });
    run("one-shot 2 x 16 B", [&] { copy_os2<<<dim3((unsigned)((n + 511) / 512)), dim3(256)>>>(s, d, n); });
    const u32x4 *sv = (const u32x4 *)s;
    u32x4 *dv = (u32x4 *)d;
    run("one-shot 1 x 16 B nt-v", [&] { copy_osv_nt<1><<<dim3((unsigned)((n + 255) / 256)), dim3(256)>>>(sv, dv, n); });
    run("one-shot 2 x 16 B nt-v", [&] { copy_osv_nt<2><<<dim3((unsigned)((n + 511) / 512)), dim3(256)>>>(sv, dv, n); });
    run("one-shot 4 x 16 B nt-v", [&] { copy_osv_nt<4><<<dim3((unsigned)((n + 1023) / 1024)), dim3(256)>>>(sv, dv, n); });
    run("one-shot 4 x 16 B nt-store", [&] { copy_os4_ntst<<<dim3((unsigned)((n + 1023) / 1024)), dim3(256)>>>(sv, dv, n); });
    run("hipMemcpyAsync D2D", [&] { CK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice)); });
    return 0;
}
