// tools/probes/exit_probe.cpp -- what a GPU process pays at exit (dev probe):
// HIP init, `pin_mb` MiB of pinned host memory (hipHostMalloc, touched),
// `dev_mb` MiB of device memory (hipMalloc), then _exit.  The caller times
// the whole process; stderr gets the in-process times.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <chrono>

int main(int argc, char** argv)
{
    const size_t pin_mb = argc > 1 ? strtoull(argv[1], nullptr, 10) : 0;
    const size_t dev_mb = argc > 2 ? strtoull(argv[2], nullptr, 10) : 0;
    const int teardown = argc > 3 ? atoi(argv[3]) : 0;
    const auto t0 = std::chrono::steady_clock::now();
    auto el = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 2;
    if (hipSetDevice(0) != hipSuccess) return 2;
    const double t_init = el();
    void* p = nullptr;
    if (pin_mb && hipHostMalloc(&p, pin_mb << 20, hipHostMallocDefault) != hipSuccess) return 3;
    if (p) memset(p, 1, pin_mb << 20);
    const double t_pin = el();
    void* d = nullptr;
    if (dev_mb && hipMalloc(&d, dev_mb << 20) != hipSuccess) return 4;
    if (d && hipMemset(d, 0, dev_mb << 20) != hipSuccess) return 4;
    if (hipDeviceSynchronize() != hipSuccess) return 5;
    const double t_dev = el();
    fprintf(stderr, "init %.3f pin %.3f dev %.3f\n", t_init, t_pin - t_init, t_dev - t_pin);
    if (teardown) {
        if (p) (void)hipHostFree(p);
        if (d) (void)hipFree(d);
        fprintf(stderr, "free %.3f\n", el() - t_dev);
        return 0;
    }
    fflush(stderr);
    _exit(0);
}
