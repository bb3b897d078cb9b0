// Memory-side u64 atomics (timing only): does the footprint of the atomics' targets set
// their rate?  16.4M atomicAdd(u64) with uniform random keys over K accounts into
//   rows  : one word of a 128-byte row per key (the account table: 128 B stride)
//   pair  : one word of a 16-byte slot per key (a dense u128 delta array)
//   dense : one 8-byte word per key
// hipcc --offload-arch=gfx950 -O3 atomics_density.hip -o atomics_density && ./atomics_density
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef unsigned long long u64;

__global__ void keys_init(unsigned* keys, unsigned n, unsigned K, u64 seed) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    u64 z = (u64)i + seed * 0x9E3779B97F4A7C15ull;
    z ^= z >> 30; z *= 0xbf58476d1ce4e5b9ull; z ^= z >> 27; z *= 0x94d049bb133111ebull; z ^= z >> 31;
    keys[i] = (unsigned)(z % K);
}
__global__ void atom(const unsigned* __restrict__ keys, u64* base, unsigned n, unsigned stride_words) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&base[(u64)keys[i] * stride_words], 1ull);
}
__global__ void atom_ret(const unsigned* __restrict__ keys, u64* base, unsigned n, unsigned stride_words, unsigned* f) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { u64 o = atomicAdd(&base[(u64)keys[i] * stride_words], 1ull); if (o == ~0ull) f[0] = 1; }
}

int main() {
    const unsigned n = 16380000;
    unsigned* keys; u64* base; unsigned* f;
    CK(hipMalloc(&keys, n * 4ull));
    CK(hipMalloc(&base, 10000000ull * 128));
    CK(hipMalloc(&f, 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (unsigned K : {1000000u, 10000000u}) {
        keys_init<<<(n + 255) / 256, 256>>>(keys, n, K, 7);
        for (unsigned stride : {16u, 2u, 1u}) {
            for (int ret = 0; ret < 2; ret++) {
                float best = 1e9;
                for (int r = 0; r < 5; r++) {
                    CK(hipEventRecord(a));
                    if (ret) atom_ret<<<(n + 255) / 256, 256>>>(keys, base, n, stride, f);
                    else atom<<<(n + 255) / 256, 256>>>(keys, base, n, stride);
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    float ms; CK(hipEventElapsedTime(&ms, a, b));
                    if (ms < best) best = ms;
                }
                printf("K=%8u stride=%3u B ret=%d: %.3f ms  %.1f G atomics/s\n", K, stride * 8, ret, best, n / best / 1e6);
            }
        }
    }
    return 0;
}
