// resident extract_kernel<true> workgroups per CU for the build flags given (occupancy API)
#include "../../dsp-audioreclabs_amd/csrc/extract.hip"
#include <cstdio>
int main()
{
    const size_t lds = extract_carve_fast().total;
    int n = -1;
    (void)hipFuncSetAttribute((const void *)dsp::extract_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, EXTRACT_LDS_LIMIT);
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dsp::extract_kernel<true>, dsp::NT, lds);
    hipFuncAttributes a;
    hipFuncGetAttributes(&a, (const void *)dsp::extract_kernel<true>);
    printf("NT %d lds %zu blocks/CU %d (err %d) regs %d localBytes %zu\n", dsp::NT, lds, n, (int)e, a.numRegs, a.localSizeBytes);
    return 0;
}
