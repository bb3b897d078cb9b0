// Does a contiguous device allocation (hipExtMallocWithFlags(hipDeviceMallocContiguous))
// alias memory of other live allocations once earlier ones have been freed?  Each live
// buffer is filled with its own tag by a kernel; after every round of allocations and
// frees, every live buffer is checked word by word.  Prints the first overlap found.
//   hipcc --offload-arch=gfx950 -O2 profiles/r04/contig_alias.hip -o contig_alias
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

__global__ void fill(unsigned* p, size_t n, unsigned tag) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = tag;
}
__global__ void check(const unsigned* p, size_t n, unsigned tag, unsigned long long* bad, unsigned* seen) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (p[i] != tag) { atomicAdd(bad, 1ull); atomicExch(seen, p[i]); }
}

struct Buf { unsigned* p; size_t words; unsigned tag; bool contig; };

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 40;
    srand(7);
    std::vector<Buf> live;
    unsigned long long* bad;
    unsigned* seen;
    CK(hipMalloc(&bad, 8));
    CK(hipMalloc(&seen, 4));
    unsigned next_tag = 1;
    const size_t sizes_mb[] = {8, 16, 32, 64, 128, 256};
    size_t overlaps = 0;
    for (int r = 0; r < rounds; r++) {
        for (int k = 0; k < 6; k++) {  // allocate: half contiguous, half plain
            Buf b;
            const size_t bytes = sizes_mb[rand() % 6] << 20;
            b.words = bytes / 4;
            b.contig = rand() & 1;
            b.tag = next_tag++;
            void* p = nullptr;
            if (b.contig) {
                if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous) != hipSuccess || !p) {
                    (void)hipGetLastError();
                    CK(hipMalloc(&p, bytes));
                    b.contig = false;
                }
            } else {
                CK(hipMalloc(&p, bytes));
            }
            b.p = (unsigned*)p;
            fill<<<1024, 256>>>(b.p, b.words, b.tag);
            live.push_back(b);
        }
        CK(hipDeviceSynchronize());
        for (const Buf& b : live) {  // every live buffer still holds its own tag
            CK(hipMemset(bad, 0, 8));
            check<<<1024, 256>>>(b.p, b.words, b.tag, bad, seen);
            unsigned long long nb = 0;
            unsigned sv = 0;
            CK(hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&sv, seen, 4, hipMemcpyDeviceToHost));
            if (nb) {
                overlaps++;
                printf("round %d: buffer tag %u (%s, %zu MB at %p) has %llu words of tag %u\n", r, b.tag,
                       b.contig ? "contiguous" : "plain", b.words * 4 >> 20, (void*)b.p, nb, sv);
            }
        }
        for (size_t k = 0; k < live.size();) {  // free about half
            if (rand() & 1) { CK(hipFree(live[k].p)); live[k] = live.back(); live.pop_back(); }
            else k++;
        }
        for (Buf& b : live) { fill<<<1024, 256>>>(b.p, b.words, b.tag); }  // refresh (an overlap rewrote one)
        CK(hipDeviceSynchronize());
    }
    printf("contig_alias: %d rounds, %zu buffers with foreign words\n", rounds, overlaps);
    return overlaps ? 1 : 0;
}
