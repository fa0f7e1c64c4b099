// Register / spill report of the ingest kernels without compiling the whole engine (VGPR spills in these kernels are
// not harmless on this toolchain: DESIGN.md section 4, "Skewed keys"). Usage:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -c tools/regprobe.hip -o /tmp/rp.o \
//         -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs|Spill"
// The instantiation list mirrors the launch sites in flink_amd/csrc/engine.hip (push_v2 and the partition launches).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../include/flink_amd.h"
#include "../flink_amd/csrc/java_math.h"

#define LONG_MIN_J ((int64_t)0x8000000000000000LL)
#define LONG_MAX_J ((int64_t)0x7fffffffffffffffLL)

namespace {
#include "../flink_amd/csrc/ingest.inc"
}  // namespace

const void* regprobe_kernels[] = {
#ifdef REGPROBE_EXTRA
    REGPROBE_EXTRA
#endif
#ifndef REGPROBE_ONLY_EXTRA
    (const void*)&combine3_kernel<2,2,0,1024,0,0,1,0>,
    (const void*)&combine3_kernel<2,2,0,1024,1,0,1,0>,
    (const void*)&combine3_kernel<2,2,0,1024,2,0,1,0>,
    (const void*)&combine3_kernel<2,2,0,1024,2,1,1,0>,
    (const void*)&combine3_kernel<2,2,1,1024,0,0,1,0>,
    (const void*)&combine3_kernel<2,2,1,1024,1,0,1,0>,
    (const void*)&combine3_kernel<2,2,1,1024,1,0,1,1>,
    (const void*)&combine3_kernel<2,2,1,1024,1,1,1,0>,
    (const void*)&combine3_kernel<2,2,1,1024,2,0,1,0>,
    (const void*)&combine3_kernel<2,2,2,1024,0,0,1,0>,
    (const void*)&combine3_kernel<2,2,2,1024,0,0,1,2>,
    (const void*)&combine3_kernel<4,2,2,1024,0,0,0,2>,
    (const void*)&partition3_kernel<2,4,1024,1,0,0,0,2>,
    (const void*)&combine3_kernel<2,2,2,1024,1,0,1,0>,
    (const void*)&combine3_kernel<2,2,2,1024,2,0,1,0>,
    (const void*)&combine3_kernel<4,2,0,1024,0,0,0,0>,
    (const void*)&combine3_kernel<4,2,0,1024,1,0,0,0>,
    (const void*)&combine3_kernel<4,2,0,1024,2,0,0,0>,
    (const void*)&combine3_kernel<4,2,0,1024,2,1,0,0>,
    (const void*)&combine3_kernel<4,2,1,1024,0,0,0,0>,
    (const void*)&combine3_kernel<4,2,1,1024,1,0,0,0>,
    (const void*)&combine3_kernel<4,2,1,1024,1,1,0,0>,
    (const void*)&combine3_kernel<4,2,1,1024,2,0,0,0>,
    (const void*)&combine3_kernel<4,2,2,1024,0,0,0,0>,
    (const void*)&combine3_kernel<4,2,2,1024,1,0,0,0>,
    (const void*)&combine3_kernel<4,2,2,1024,2,0,0,0>,
    (const void*)&combine3_kernel<6,2,1,1024,1,0,0,1>,
    (const void*)&partition3_kernel<0,4,1024,3,0,1,0,0>,
    (const void*)&partition3_kernel<0,4,1024,3,1,1,0,0>,
    (const void*)&partition3_kernel<0,4,1024,3,2,1,0,0>,
    (const void*)&partition3_kernel<0,8,1024,3,0,0,0,0>,
    (const void*)&partition3_kernel<0,8,1024,3,1,0,0,0>,
    (const void*)&partition3_kernel<0,8,1024,3,2,0,0,0>,
    (const void*)&partition3_kernel<1,4,1024,3,0,1,0,0>,
    (const void*)&partition3_kernel<1,4,1024,3,1,1,0,0>,
    (const void*)&partition3_kernel<1,4,1024,3,2,1,0,0>,
    (const void*)&partition3_kernel<1,6,1024,2,0,0,0,0>,
    (const void*)&partition3_kernel<1,6,1024,2,0,0,1,0>,
    (const void*)&partition3_kernel<1,6,1024,2,1,0,0,0>,
    (const void*)&partition3_kernel<1,6,1024,2,2,0,0,0>,
    (const void*)&partition3_kernel<1,6,1024,3,0,0,0,0>,
    (const void*)&partition3_kernel<1,6,1024,3,0,0,1,0>,
    (const void*)&partition3_kernel<1,6,1024,3,0,0,1,1>,
    (const void*)&partition3_kernel<1,6,1024,3,1,0,0,0>,
    (const void*)&partition3_kernel<1,6,1024,3,2,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,0,0,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,0,1,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,0,2,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,1,0,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,1,1,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,1,2,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,2,0,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,2,1,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,2,2,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,3,0,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,3,1,0,0,0>,
    (const void*)&partition3_kernel<2,4,1024,3,2,0,0,0>,
#endif
};
