// Probe: cost of a cooperative-groups grid barrier on MI355X for small grids (the radix sort's
// 66-256 tiles): one cooperative launch, R grid.sync() calls, timed with HIP events.
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <cstdio>
#include <cstdlib>

namespace cg = cooperative_groups;

__global__ void sync_loop(int reps, unsigned* sink) {
    cg::grid_group grid = cg::this_grid();
    unsigned acc = 0;
    for (int r = 0; r < reps; ++r) {
        acc += blockIdx.x + r;
        grid.sync();
    }
    if (threadIdx.x == 0 && acc == 0xdeadbeef) sink[0] = acc;
}

int main(int argc, char** argv) {
    const int grids[] = {66, 83, 128, 256};
    unsigned* sink = nullptr;
    if (hipMalloc(&sink, 64) != hipSuccess) return 1;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int g : grids) {
        for (int reps : {1, 101}) {
            void* args[] = {&reps, &sink};
            // warm-up
            if (hipLaunchCooperativeKernel((void*)sync_loop, dim3(g), dim3(256), args, 0, 0) != hipSuccess) {
                printf("{\"grid\": %d, \"error\": \"cooperative launch failed\"}\n", g);
                return 2;
            }
            hipDeviceSynchronize();
            hipEventRecord(a, 0);
            for (int i = 0; i < 10; ++i) hipLaunchCooperativeKernel((void*)sync_loop, dim3(g), dim3(256), args, 0, 0);
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            printf("{\"grid\": %d, \"syncs\": %d, \"us_per_launch\": %.3f}\n", g, reps, ms * 1e3 / 10);
        }
    }
    return 0;
}
