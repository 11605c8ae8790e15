// hip_emu.cpp -- TEST INFRASTRUCTURE ONLY: block scheduler of the CPU emulator.
#include "hip_emu.h"

#include <memory>

thread_local emu_idx threadIdx, blockIdx;
emu_idx blockDim, gridDim;
emu_block_sync *g_emu_sync = nullptr;

void emu_run_grid(dim3 grid, dim3 block, const std::function<void()> &body) {
    const unsigned nt = block.x * block.y * block.z;
    blockDim = {block.x, block.y, block.z};
    gridDim = {grid.x, grid.y, grid.z};
    emu_block_sync sync;
    std::barrier<> bar((std::ptrdiff_t)nt);
    sync.bar = &bar;
    sync.xch.assign(nt, 0);
    std::vector<std::unique_ptr<std::barrier<>>> wbars;
    for (unsigned w = 0; w * 64 < nt; w++) {
        wbars.emplace_back(new std::barrier<>((std::ptrdiff_t)std::min(64u, nt - w * 64)));
        sync.wave_bar.push_back(wbars.back().get());
    }
    g_emu_sync = &sync;
    const unsigned long long nb = (unsigned long long)grid.x * grid.y * grid.z;
    // persistent workers: one per thread of the block, all walking the blocks
    std::vector<std::thread> workers;
    workers.reserve(nt);
    for (unsigned t = 0; t < nt; t++) {
        workers.emplace_back([&, t]() {
            threadIdx = {t, 0, 0};
            for (unsigned long long b = 0; b < nb; b++) {
                blockIdx = {(unsigned)b, 0, 0};
                body();
                bar.arrive_and_wait();  // block boundary (also covers early returns)
            }
        });
    }
    for (auto &w : workers) w.join();
    g_emu_sync = nullptr;
}
