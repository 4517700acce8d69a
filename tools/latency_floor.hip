// Round-trip floor of one tiny kernel on this box: launch + completion seen by the host, with the
// synchronisation styles the small host batch could use (tools/README.md). Build:
//   hipcc --offload-arch=gfx950 -O2 -o tools/latency_floor tools/latency_floor.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void touch(uint32_t* p) { p[threadIdx.x] += 1; }

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    uint32_t* h;
    hipHostMalloc((void**)&h, 4096, hipHostMallocMapped);
    uint32_t* d;
    hipHostGetDevicePointer((void**)&d, h, 0);
    hipEvent_t ev, e0;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    hipEventCreateWithFlags(&e0, hipEventDisableTiming);
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    const char* names[] = {"launch+streamSync", "launch+spin(streamQuery)", "launch+event+spin(eventQuery)",
                           "nullEvent+wait+launch+streamSync", "launch+spin(host flag)"};
    for (int mode = 0; mode < 5; mode++) {
        std::vector<double> us;
        for (int r = 0; r < 3000; r++) {
            const uint32_t before = h[0];
            const auto a = std::chrono::steady_clock::now();
            if (mode == 3) {
                hipEventRecord(e0, nullptr);
                hipStreamWaitEvent(s, e0, 0);
            }
            hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, s, d);
            if (mode == 0 || mode == 3) hipStreamSynchronize(s);
            else if (mode == 1) while (hipStreamQuery(s) == hipErrorNotReady) {}
            else if (mode == 2) { hipEventRecord(ev, s); while (hipEventQuery(ev) == hipErrorNotReady) {} }
            else { while (__atomic_load_n(&h[0], __ATOMIC_ACQUIRE) == before) {} hipStreamSynchronize(s); }
            us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
        }
        std::printf("%-36s median %.2f us\n", names[mode], med(us));
    }
    return 0;
}
