// Single-kernel resource build (development): the registers, spills and scratch of one layer kernel
// in seconds, without compiling the whole library.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -c -Rpass-analysis=kernel-resource-usage \
//       -DKDEV_INST='template __global__ void k_dgrad<1, 16, 4, 2, true, 1>(BwdArgs);' tools/kdev.hip -o /tmp/kdev.o
#include "../3d-pose-baseline_amd/csrc/p3d_layers.h"
#ifndef KDEV_INST
#define KDEV_INST template __global__ void k_dgrad<1, 16, 4, 2, true, 1>(BwdArgs);
#endif
KDEV_INST
