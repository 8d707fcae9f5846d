// HBM ceilings for the streaming kernel's traffic mix (timing probe, not product).
//
// Round 4 rewrite: every lane keeps U independent 16-byte loads in flight (unrolled, the loads of
// one iteration issued before any use), blocks walk contiguous chunks (not a grid-stride loop of
// one load per lane), buffers far larger than the 256 MiB Infinity Cache; HIP events, best of 10.
// Lines: read-only, write-only (dwordx4 per lane, and the streaming kernel's own store shape --
// 12 bytes per lane as three dword stores and as one dwordx3), read + write copies, plain and
// nontemporal.  Usage: copy_probe [MiB per buffer, default 1300].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v3u __attribute__((ext_vector_type(3)));

constexpr int kThreads = 256;

// Block b owns elements [b * per, (b + 1) * per); per iteration each lane touches U elements
// kThreads apart (each wave-instruction = 1 KiB contiguous).
template <int U, int NT>
__global__ __launch_bounds__(kThreads) void read_k(const v4u *__restrict__ a, unsigned *out,
                                                   size_t per)
{
    const v4u *p = a + blockIdx.x * per + threadIdx.x;
    v4u s = {0, 0, 0, 0};
    for (size_t i = 0; i < per; i += (size_t)U * kThreads) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(p + i + u * kThreads)
                                              : p[i + u * kThreads];
#pragma unroll
        for (int u = 0; u < U; u++) s ^= v[u];
    }
    if ((s.x ^ s.y ^ s.z ^ s.w) == 0x12345678u) out[0] = 1;
}

template <int U, int NT>
__global__ __launch_bounds__(kThreads) void write_k(v4u *__restrict__ b, size_t per)
{
    v4u *p = b + blockIdx.x * per + threadIdx.x;
    const v4u v = {1u, 2u, 3u, (unsigned)threadIdx.x};
    for (size_t i = 0; i < per; i += (size_t)U * kThreads) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (NT) __builtin_nontemporal_store(v, p + i + u * kThreads);
            else p[i + u * kThreads] = v;
        }
    }
}

// The streaming kernel's store shape: 12 bytes per lane, lanes contiguous (768 B per
// wave-instruction group).  FORM 0: three dword stores (the current kernel); 1: one dwordx3.
template <int FORM, int NT>
__global__ __launch_bounds__(kThreads) void write12_k(unsigned *__restrict__ b, size_t per_lanes)
{
    const size_t base = ((size_t)blockIdx.x * per_lanes + threadIdx.x) * 3;
    for (size_t i = 0; i < per_lanes; i += kThreads) {
        unsigned *o = b + base + i * 3;
        if (FORM == 0) {
            if (NT) {
                __builtin_nontemporal_store(1u, o);
                __builtin_nontemporal_store(2u, o + 1);
                __builtin_nontemporal_store(3u, o + 2);
            } else {
                o[0] = 1u;
                o[1] = 2u;
                o[2] = 3u;
            }
        } else {
            const v3u v = {1u, 2u, 3u};
            if (NT) __builtin_nontemporal_store(v, reinterpret_cast<v3u *>(o));
            else *reinterpret_cast<v3u *>(o) = v;
        }
    }
}

template <int U, int NT_LOAD, int NT_STORE>
__global__ __launch_bounds__(kThreads) void copy_k(const v4u *__restrict__ a, v4u *__restrict__ b,
                                                   size_t per)
{
    const size_t o = blockIdx.x * per + threadIdx.x;
    for (size_t i = 0; i < per; i += (size_t)U * kThreads) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = NT_LOAD ? __builtin_nontemporal_load(a + o + i + u * kThreads)
                                                   : a[o + i + u * kThreads];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (NT_STORE) __builtin_nontemporal_store(v[u], b + o + i + u * kThreads);
            else b[o + i + u * kThreads] = v[u];
        }
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <class F>
float best(F f)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    CK(hipDeviceSynchronize());
    float b = 1e30f;
    for (int r = 0; r < 10; r++) {
        CK(hipEventRecord(e0));
        f();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        b = ms < b ? ms : b;
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return b;
}

int main(int argc, char **argv)
{
    const size_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1300;
    const size_t unit = (size_t)16 * kThreads * 8;         // one block iteration at U = 8 (32 KiB)
    v4u *a, *b;
    unsigned *o;
    const size_t cap = (mib << 20) / unit * unit;
    CK(hipMalloc(&a, cap));
    CK(hipMalloc(&b, cap));
    CK(hipMalloc(&o, 4));
    CK(hipMemset(a, 1, cap));
    CK(hipMemset(b, 2, cap));
    printf("buffers %zu MiB each\n", cap >> 20);
    for (int blocks : {2048, 4096, 8192}) {
        // bytes per block: a multiple of one U = 8 iteration, so every U divides it
        const size_t per_b = cap / blocks / unit * unit, bytes = per_b * blocks, per = per_b / 16;
        auto gbs = [&](float ms, double mult) { return mult * (double)bytes / ms / 1e6; };
        float t;
#define LINE(label, mult, launch)                                                                  \
    t = best([&] { launch; });                                                                     \
    printf("blocks %5d %-24s %.4f ms %6.0f GB/s\n", blocks, label, t, gbs(t, mult));
        LINE("read U1", 1, (read_k<1, 0><<<blocks, kThreads>>>(a, o, per)));
        LINE("read U4", 1, (read_k<4, 0><<<blocks, kThreads>>>(a, o, per)));
        LINE("read U8", 1, (read_k<8, 0><<<blocks, kThreads>>>(a, o, per)));
        LINE("read U8 nt", 1, (read_k<8, 1><<<blocks, kThreads>>>(a, o, per)));
        LINE("write U1", 1, (write_k<1, 0><<<blocks, kThreads>>>(b, per)));
        LINE("write U8", 1, (write_k<8, 0><<<blocks, kThreads>>>(b, per)));
        LINE("write U8 nt", 1, (write_k<8, 1><<<blocks, kThreads>>>(b, per)));
        const size_t lanes = per_b / 12 / kThreads * kThreads;   // 12-B lanes per block
        const double f12 = (double)(lanes * 12) / (double)per_b;
        LINE("write 12B 3xdword", f12, (write12_k<0, 0><<<blocks, kThreads>>>((unsigned *)b, lanes)));
        LINE("write 12B 3xdword nt", f12, (write12_k<0, 1><<<blocks, kThreads>>>((unsigned *)b, lanes)));
        LINE("write 12B dwordx3", f12, (write12_k<1, 0><<<blocks, kThreads>>>((unsigned *)b, lanes)));
        LINE("write 12B dwordx3 nt", f12, (write12_k<1, 1><<<blocks, kThreads>>>((unsigned *)b, lanes)));
        LINE("copy U1 (r+w)", 2, (copy_k<1, 0, 0><<<blocks, kThreads>>>(a, b, per)));
        LINE("copy U4 (r+w)", 2, (copy_k<4, 0, 0><<<blocks, kThreads>>>(a, b, per)));
        LINE("copy U8 (r+w)", 2, (copy_k<8, 0, 0><<<blocks, kThreads>>>(a, b, per)));
        LINE("copy U8 nt-store (r+w)", 2, (copy_k<8, 0, 1><<<blocks, kThreads>>>(a, b, per)));
        LINE("copy U8 nt both (r+w)", 2, (copy_k<8, 1, 1><<<blocks, kThreads>>>(a, b, per)));
#undef LINE
    }
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(o));
    return 0;
}
