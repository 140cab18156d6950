// dup_fetch_probe.hip -- does one wave-wide global_load_dwordx4 whose lanes share addresses
// fetch a shared 16-byte chunk once (per cache line), or once per lane?  (VERDICT r05 item 1b:
// the list kernel's slab G ops, whose P paths read through a slot table -- several lanes of a
// codeword group often read the same slot's column.)
//
// Layout as the list kernel's slab: chunk c of "column" l at ((c * 64) + l) * 16 B.  Lane l of a
// wave reads column src(l) for every chunk of its wave's private region (larger than L2 in
// total, read once: every line comes from beyond L2).  Patterns:
//   0  src(l) = l                          (all distinct: 1 KiB of unique data per instruction)
//   1  src(l) = l & ~1                     (adjacent pairs share)
//   2  src(l) = (l & ~7) | perm[l & 7]     (8-lane groups, 4 distinct slots, scattered lanes)
//   3  src(l) = l & ~7                     (every 8-lane group reads one slot)
// Run each pattern under `rocprofv3 --pmc FETCH_SIZE`; compare with the unique bytes printed.
// Measured (profiles/r06d_dup_fetch_probe.txt): all four patterns fetch the same 537 MB per
// launch (FETCH_SIZE x 2, the gfx950 correction) = 8 lines x 128 B per instruction -- fetches are
// per 128-B line and instruction.  In the slab layout the 8 path columns of a codeword group for
// one chunk ARE one 128-B line, so a G reading any mix of slots fetches exactly that line: there
// are no duplicate slot reads to remove.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void __launch_bounds__(64) probe(const float4* __restrict__ slab, float* out, int pattern, int chunks)
{
    const unsigned l = threadIdx.x;
    const unsigned perm[8] = { 0, 0, 3, 3, 5, 5, 5, 6 };
    unsigned src = l;
    if (pattern == 1)
        src = l & ~1u;
    else if (pattern == 2)
        src = (l & ~7u) | perm[l & 7u];
    else if (pattern == 3)
        src = l & ~7u;
    const float4* b = slab + (size_t)blockIdx.x * chunks * 64;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int c = 0; c < chunks; ++c) {
        const float4 v = b[(size_t)c * 64 + src];
        acc.x += v.x;
        acc.y += v.y;
        acc.z += v.z;
        acc.w += v.w;
    }
    out[blockIdx.x * 64 + l] = acc.x + acc.y + acc.z + acc.w;
}

int main(int argc, char** argv)
{
    const int pattern = argc > 1 ? atoi(argv[1]) : 0;
    const int waves = 8192, chunks = 64; // 8192 waves x 64 KiB = 512 MiB region, read once
    float4* slab;
    float* out;
    const size_t n = (size_t)waves * chunks * 64;
    if (hipMalloc(&slab, n * sizeof(float4)) != hipSuccess || hipMalloc(&out, (size_t)waves * 64 * 4) != hipSuccess)
        return 1;
    (void)hipMemset(slab, 0, n * sizeof(float4));
    for (int it = 0; it < 2; ++it)
        hipLaunchKernelGGL(probe, dim3(waves), dim3(64), 0, 0, slab, out, pattern, chunks);
    if (hipDeviceSynchronize() != hipSuccess)
        return 2;
    const double distinct = pattern == 0 ? 64 : pattern == 1 ? 32 : pattern == 2 ? 32 : 8;
    printf("pattern %d: requested %.0f B per launch (every lane), unique %.0f B per launch\n", pattern,
           (double)waves * chunks * 64 * 16, (double)waves * chunks * distinct * 16);
    return 0;
}
