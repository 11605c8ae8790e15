// Test infrastructure only: shadows <hip/hip_runtime.h> when grom_amd's HIP
// sources are compiled for the CPU emulator (tests/emu/Makefile).
#include "../hip_emu.h"
