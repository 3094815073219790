// XCD-aware block order (shared by the MNIST and CIFAR10 kernels).  Workgroups are dealt round-robin over the 8
// XCDs (block b and b + 8 share one, MI355X_MICROARCH.md), so a replica's consecutive blocks would land on all 8
// XCDs and each XCD's L2 would fetch that replica's weights.  The flat block id is remapped so that each XCD walks a
// contiguous range of logical blocks (replica-major when the replica is the outermost grid dimension): the blocks
// of one replica share an XCD and its L2.  The mapping only permutes which workgroup does which tile of work;
// every result is bit-identical.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ int64_t xcd_block() {
  const int64_t n = (int64_t)gridDim.x * gridDim.y * gridDim.z;
  const int64_t b = blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z);
  const int64_t q = n / 8;
  return b < 8 * q ? (b % 8) * q + b / 8 : b;
}

// the logical block's (x, y, z) in the launch grid's shape
struct LogicalBlock {
  int x, y, z;
};
__device__ __forceinline__ LogicalBlock xcd_block3() {
  const int64_t lb = xcd_block();
  const int64_t t = lb / gridDim.x;
  return LogicalBlock{(int)(lb % gridDim.x), (int)(t % gridDim.y), (int)(t / gridDim.y)};
}

}  // namespace
