// k_asm.hip — file assembly of one job in HBM: the Thrift page headers (built on the host,
// filewriter.cpp) and the compressed page bodies (already in HBM) are gathered into the byte
// order of the file, so one DMA lands the job's row groups in the in-memory file and no host
// thread copies page bodies.  One workgroup per piece of <= 64 KiB.
#include "kpw_device.h"
#include "kpw_kernels.h"

namespace kpw {

__global__ void __launch_bounds__(256) k_asm_gather(const AsmPiece *pc, const uint8_t *blob, uint8_t *out)
{
    const AsmPiece P = pc[blockIdx.x];
    const uint8_t *src = P.dev ? (const uint8_t *)(uintptr_t)P.src : blob + P.src;
    block_copy(out + P.dst, src, P.len, threadIdx.x, 256);
}

void launch_asm_gather(const AsmPiece *pc, uint32_t npieces, const uint8_t *blob, uint8_t *out, hipStream_t s)
{
    if (npieces) hipLaunchKernelGGL(k_asm_gather, dim3(npieces), dim3(256), 0, s, pc, blob, out);
}

}  // namespace kpw
