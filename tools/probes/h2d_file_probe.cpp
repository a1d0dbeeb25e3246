// tools/probes/h2d_file_probe.cpp -- ways to move a page-cached file into HBM
// (dev probe for the CLI's file path): argv[1] = file.  Prints GB/s of
//   pageable   hipMemcpy from the file's mmap (runtime staging)
//   register   hipHostRegister of the mmap (cost), then hipMemcpy from it
//   staged     16 threads memcpy mmap -> two 64 MiB pinned buffers, async H2D
//   pread      16 threads pread -> two 64 MiB pinned buffers, async H2D
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <thread>
#include <vector>

#define CK(x) do { if ((x) != hipSuccess) { fprintf(stderr, "%s failed\n", #x); return 1; } } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv)
{
    if (argc < 2) return 2;
    const int fd = open(argv[1], O_RDONLY);
    struct stat sb;
    if (fd < 0 || fstat(fd, &sb)) return 2;
    const size_t n = (size_t)sb.st_size;
    CK(hipSetDevice(0));
    void* d = nullptr;
    CK(hipMalloc(&d, n));
    hipStream_t st[2];
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int T = 16;
    auto par = [&](size_t len, auto fn) {
        std::vector<std::thread> th;
        const size_t per = (len + T - 1) / T;
        for (int t = 0; t < T; ++t) th.emplace_back([&, t]() { const size_t a = t * per, b = std::min(len, a + per); if (a < b) fn(a, b); });
        for (auto& x : th) x.join();
    };
    {   // pageable from a fresh mmap
        void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        double t = now();
        CK(hipMemcpy(d, m, n, hipMemcpyHostToDevice));
        t = now() - t;
        printf("pageable mmap hipMemcpy: %.1f ms %.1f GB/s\n", t * 1e3, n / t / 1e9);
        t = now();
        CK(hipMemcpy(d, m, n, hipMemcpyHostToDevice));
        t = now() - t;
        printf("pageable mmap hipMemcpy (mapped): %.1f ms %.1f GB/s\n", t * 1e3, n / t / 1e9);
        munmap(m, n);
    }
    {   // register the mmap
        void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        double t = now();
        const hipError_t e = hipHostRegister(m, n, hipHostRegisterReadOnly);
        const double tr = now() - t;
        if (e == hipSuccess) {
            t = now();
            CK(hipMemcpy(d, m, n, hipMemcpyHostToDevice));
            t = now() - t;
            printf("register %.1f ms; registered hipMemcpy %.1f ms %.1f GB/s\n", tr * 1e3, t * 1e3, n / t / 1e9);
            t = now();
            (void)hipHostUnregister(m);
            printf("unregister %.1f ms\n", (now() - t) * 1e3);
        } else {
            printf("hipHostRegister failed (%d) after %.1f ms\n", (int)e, tr * 1e3);
        }
        munmap(m, n);
    }
    const size_t B = 64ull << 20;
    void* pin[2];
    double tp = now();
    for (auto& p : pin) CK(hipHostMalloc(&p, B, hipHostMallocDefault));
    printf("pin 2 x 64 MiB: %.1f ms\n", (now() - tp) * 1e3);
    hipEvent_t ev[2];
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (int mode = 0; mode < 2; ++mode) {
        void* m = mode == 0 ? mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
        double t = now();
        for (size_t off = 0, k = 0; off < n; off += B, ++k) {
            const int b = (int)(k & 1);
            const size_t len = std::min(B, n - off);
            CK(hipEventSynchronize(ev[b]));
            if (mode == 0) par(len, [&](size_t a, size_t e) { memcpy((char*)pin[b] + a, (char*)m + off + a, e - a); });
            else par(len, [&](size_t a, size_t e) { size_t q = a; while (q < e) { ssize_t r = pread(fd, (char*)pin[b] + q, e - q, off + q); if (r <= 0) break; q += r; } });
            CK(hipMemcpyAsync((char*)d + off, pin[b], len, hipMemcpyHostToDevice, st[b]));
            CK(hipEventRecord(ev[b], st[b]));
        }
        CK(hipDeviceSynchronize());
        t = now() - t;
        printf("%s -> 2 x 64 MiB pinned -> H2D: %.1f ms %.1f GB/s\n", mode == 0 ? "mmap memcpy" : "pread", t * 1e3, n / t / 1e9);
        if (m) munmap(m, n);
    }
    return 0;
}
