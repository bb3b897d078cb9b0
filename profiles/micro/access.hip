// Access-pattern floor for fp_commit's memory shapes (timing only):
//   copy_strided   : one 128-B event per lane (8 x 16-B loads at 128-B lane stride), row store
//   copy_coalesced : the same bytes, 16 B per lane consecutive (wave = 1 KiB per instruction)
//   probe2         : strided event read + two dependent 32-B index reads (64 MB table, Zipf-ish keys)
//   atomics        : one 8-B atomic per lane into random 128-B rows of a 128 MB table
// hipcc --offload-arch=gfx950 -O3 access.hip -o access && ./access
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef unsigned long long u64;
struct alignas(16) Ev { uint4 q[8]; };
struct alignas(32) Idx { u64 a, b; unsigned r, l, f, c; };

__global__ void copy_strided(const Ev* __restrict__ in, Ev* __restrict__ out, unsigned n) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { Ev e = in[i]; e.q[7].w += 1; out[i] = e; }
}
__global__ void copy_coalesced(const uint4* __restrict__ in, uint4* __restrict__ out, unsigned n16) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n16) { uint4 v = in[i]; if ((i & 7) == 7) v.w += 1; out[i] = v; }
}
__global__ void probe2(const Ev* __restrict__ in, const Idx* __restrict__ idx, u64 mask, unsigned* out, unsigned n) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ev e = in[i];
    u64 h1 = (((u64)e.q[1].x << 32) | e.q[1].y) * 0x9E3779B97F4A7C15ull;
    u64 h2 = (((u64)e.q[2].x << 32) | e.q[2].y) * 0x9E3779B97F4A7C15ull;
    Idx A = idx[(h1 >> 20) & mask], B = idx[(h2 >> 20) & mask];
    out[i] = A.r + B.r + e.q[3].x;
}
__global__ void atomics(const unsigned* __restrict__ keys, u64* rows, unsigned n) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&rows[(u64)keys[i] * 16 + 2], 1ull);
}
__global__ void atomics_at(const u64* __restrict__ at, u64* base, unsigned n) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&base[at[i]], 1ull);
}
__global__ void atomics_ret(const unsigned* __restrict__ keys, u64* rows, unsigned n, unsigned* flag) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { u64 o = atomicAdd(&rows[(u64)keys[i] * 16 + 2], 1ull); if (o == ~0ull) flag[0] = 1; }
}

__global__ void init_ev(Ev* in, unsigned n) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int k = 0; k < 8; k++) {
        u64 z = (u64)i * 8 + k + 0x9E3779B97F4A7C15ull; z ^= z >> 30; z *= 0xbf58476d1ce4e5b9ull; z ^= z >> 27; z *= 0x94d049bb133111ebull; z ^= z >> 31;
        in[i].q[k] = make_uint4((unsigned)z, (unsigned)(z >> 32), (unsigned)(z * 3), (unsigned)(z >> 7));
    }
}

// (c) strided load -> LDS transpose -> coalesced row store
__global__ __launch_bounds__(256) void copy_lds_out(const Ev* __restrict__ in, Ev* __restrict__ out, unsigned* o32, unsigned n) {
    __shared__ uint4 s[4][64 * 8];
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    Ev e = in[i];
    for (int k = 0; k < 8; k++) s[w][lane * 8 + k] = e.q[k];
    __builtin_amdgcn_wave_barrier();
    const unsigned base = (blockIdx.x * blockDim.x + w * 64) * 8;
    for (int k = 0; k < 8; k++) { uint4 v = s[w][k * 64 + lane]; if ((lane & 7) == 7) v.w += 1; ((uint4*)out)[base + k * 64 + lane] = v; }
    o32[i] = e.q[1].x + e.q[3].y;
}
// (d) coalesced load -> coalesced row store + LDS -> per-lane event
__global__ __launch_bounds__(256) void copy_lds_in(const Ev* __restrict__ in, Ev* __restrict__ out, unsigned* o32, unsigned n) {
    __shared__ uint4 s[4][64 * 8];
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned base = (blockIdx.x * blockDim.x + w * 64) * 8;
    uint4 v[8];
    for (int k = 0; k < 8; k++) v[k] = ((const uint4*)in)[base + k * 64 + lane];
    for (int k = 0; k < 8; k++) { s[w][k * 64 + lane] = v[k]; if ((lane & 7) == 7) v[k].w += 1; ((uint4*)out)[base + k * 64 + lane] = v[k]; }
    __builtin_amdgcn_wave_barrier();
    Ev e;
    for (int k = 0; k < 8; k++) e.q[k] = s[w][lane * 8 + k];
    o32[i] = e.q[1].x + e.q[3].y + e.q[7].z;
}
// (e) coalesced load + store, then per-lane strided re-read (cache hits)
__global__ __launch_bounds__(256) void copy_reread(const Ev* __restrict__ in, Ev* __restrict__ out, unsigned* o32, unsigned n) {
    const unsigned lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned base = (blockIdx.x * blockDim.x + w * 64) * 8;
    uint4 v[8];
    for (int k = 0; k < 8; k++) v[k] = ((const uint4*)in)[base + k * 64 + lane];
    for (int k = 0; k < 8; k++) { if ((lane & 7) == 7) v[k].w += 1; ((uint4*)out)[base + k * 64 + lane] = v[k]; }
    Ev e = in[i];
    o32[i] = e.q[1].x + e.q[3].y + e.q[7].z;
}
// strided load with the row store, fields used (the current fp_commit shape)
__global__ __launch_bounds__(256) void copy_strided_use(const Ev* __restrict__ in, Ev* __restrict__ out, unsigned* o32, unsigned n) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    Ev e = in[i];
    o32[i] = e.q[1].x + e.q[3].y + e.q[7].z;
    e.q[7].w += 1; out[i] = e;
}

int main() {
    const unsigned n = 1638400, accounts = 1 << 20;
    Ev *in, *out; Idx* idx; unsigned *keys, *o32; u64* rows;
    CK(hipMalloc(&in, (size_t)n * 128)); CK(hipMalloc(&out, (size_t)n * 128));
    CK(hipMalloc(&idx, (size_t)2 * accounts * 32)); CK(hipMalloc(&keys, (size_t)n * 4 * 2));
    CK(hipMalloc(&o32, (size_t)n * 4)); CK(hipMalloc(&rows, (size_t)accounts * 128));
    std::vector<unsigned> hk(2 * n), hz(2 * n); srand(1);
    for (auto& k : hk) k = (unsigned)(((u64)rand() << 16 ^ rand()) % accounts);
    {   // Zipf(0.99) ranks over 1M accounts, rank -> row by a fixed permutation
        std::vector<double> cdf(accounts); double acc = 0;
        for (unsigned r = 0; r < accounts; r++) { acc += pow(r + 1.0, -0.99); cdf[r] = acc; }
        std::vector<unsigned> perm(accounts); for (unsigned r = 0; r < accounts; r++) perm[r] = r;
        for (unsigned r = accounts - 1; r > 0; r--) std::swap(perm[r], perm[((u64)rand() << 16 ^ rand()) % (r + 1)]);
        for (auto& k : hz) { double u = (double)(((u64)rand() << 16) ^ rand()) / (double)(1ull << 47) * acc;
            k = perm[std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin()]; }
    }
    unsigned* zkeys; CK(hipMalloc(&zkeys, (size_t)n * 4 * 2));
    CK(hipMemcpy(keys, hk.data(), hk.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(zkeys, hz.data(), hz.size() * 4, hipMemcpyHostToDevice));
    // the fp_commit flush pattern: per 512-event tile, one atomic per distinct key
    // (dr keys and cr keys are different fields); variants replicate the keys that
    // occur >= 2 times in the tile over R stripes chosen by tile % R
    std::vector<u64> fl[4]; const int RS[4] = {1, 8, 64, 0};
    for (unsigned t = 0; t < n / 512; t++) {
        std::vector<std::pair<unsigned, unsigned>> ks;
        for (unsigned e = t * 512; e < t * 512 + 512; e++) { ks.push_back({hz[2 * e] * 4 + 1, 0}); ks.push_back({hz[2 * e + 1] * 4 + 3, 0}); }
        std::sort(ks.begin(), ks.end());
        for (size_t a = 0; a < ks.size();) { size_t b = a; while (b < ks.size() && ks[b].first == ks[a].first) b++;
            const bool hot = b - a >= 2;
            for (int v = 0; v < 4; v++) {
                if (v == 3) { if (!hot) fl[v].push_back((u64)ks[a].first * 2); continue; }  // cold only
                u64 addr = (u64)ks[a].first * 2;                           // u64 word of the field
                if (hot && RS[v] > 1) addr = (u64)accounts * 16 + ((u64)(t % RS[v]) * accounts * 4 + ks[a].first) ;
                fl[v].push_back(addr);
            }
            a = b; }
    }
    u64* big; CK(hipMalloc(&big, (size_t)accounts * 16 * 8 + (size_t)64 * accounts * 4 * 8));
    u64* fla[4];
    for (int v = 0; v < 4; v++) { CK(hipMalloc(&fla[v], fl[v].size() * 8)); CK(hipMemcpy(fla[v], fl[v].data(), fl[v].size() * 8, hipMemcpyHostToDevice)); }
    printf("flush atomics per tile-aggregated call: %zu (cold only %zu)\n", fl[0].size(), fl[3].size());
    unsigned* k10; CK(hipMalloc(&k10, (size_t)n * 4 * 2));
    for (auto& k : hk) k %= 10000;
    CK(hipMemcpy(k10, hk.data(), hk.size() * 4, hipMemcpyHostToDevice));
    init_ev<<<(n + 255) / 256, 256>>>(in, n); CK(hipMemset(idx, 0, (size_t)2 * accounts * 32)); CK(hipMemset(rows, 0, (size_t)accounts * 128));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto run = [&](const char* name, double bytes, auto f) {
        for (int w = 0; w < 3; w++) f();
        CK(hipEventRecord(a)); for (int r = 0; r < 10; r++) f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); ms /= 10;
        printf("%-16s %8.4f ms  %7.1f GB/s  %6.2f ns/1k-ev\n", name, ms, bytes / ms / 1e6, ms * 1e6 / n * 1e3 / 1e3);
    };
    run("strided_use", 256.0 * n, [&] { copy_strided_use<<<n / 256, 256>>>(in, out, o32, n); });
    run("lds_out", 256.0 * n, [&] { copy_lds_out<<<n / 256, 256>>>(in, out, o32, n); });
    run("lds_in", 256.0 * n, [&] { copy_lds_in<<<n / 256, 256>>>(in, out, o32, n); });
    run("reread", 256.0 * n, [&] { copy_reread<<<n / 256, 256>>>(in, out, o32, n); });
    for (int bs : {256}) {
        printf("block %d\n", bs);
        run("copy_strided", 256.0 * n, [&] { copy_strided<<<(n + bs - 1) / bs, bs>>>(in, out, n); });
        run("copy_coalesced", 256.0 * n, [&] { copy_coalesced<<<(n * 8 + bs - 1) / bs, bs>>>((const uint4*)in, (uint4*)out, n * 8); });
        run("probe2", 128.0 * n, [&] { probe2<<<(n + bs - 1) / bs, bs>>>(in, idx, 2 * accounts - 1, o32, n); });
        run("atomics 2/ev", 0, [&] { atomics<<<(2 * n + bs - 1) / bs, bs>>>(keys, rows, 2 * n); });
        run("atomics zipf", 0, [&] { atomics<<<(2 * n + bs - 1) / bs, bs>>>(zkeys, rows, 2 * n); });
        run("atomics 10k", 0, [&] { atomics<<<(2 * n + bs - 1) / bs, bs>>>(k10, rows, 2 * n); });
        for (int v = 0; v < 4; v++) {
            char nm[64]; snprintf(nm, 64, v == 3 ? "flush cold only" : "flush R=%d", RS[v]);
            const unsigned m = fl[v].size();
            run(nm, 0, [&] { atomics_at<<<(m + bs - 1) / bs, bs>>>(fla[v], big, m); });
        }
        run("atomics_ret 2/ev", 0, [&] { atomics_ret<<<(2 * n + bs - 1) / bs, bs>>>(keys, rows, 2 * n, o32); });
    }
    return 0;
}
