// lfa_probe.hip — the reduce_tree_put wrong-result probe,
// built into liblfa_tune.so only.  lfa__tp_probe(form, ...) launches the
// int8 FI_SUM vector body at 16 leaves with 4 KiB tiles per wave — the
// instantiation that round 2 found wrong — in four register regimes:
//   form 0  the round-2 kernel (wave index divergent to the compiler:
//           buffer accesses in readfirstlane loops), 278 registers per lane:
//           256 VGPRs + 22 AGPRs holding live values
//   form 1  the round-3 kernel (wave index readfirstlane'd: scalar tiles),
//           256 VGPRs + 20 AGPRs
//   form 2  form 1's body limited to 256 registers per lane
//           (amdgpu_waves_per_eu(2, 2)): no AGPR holds a value, the excess
//           spills to scratch memory (84 B per lane)
//   form 3  form 0's body limited likewise (100 B per lane of scratch)
// tools/probe_treeput_narrow.py --probe compares each lane by lane with the
// oracle.  Vector body only: nsrc 16..31 inputs, cnt a multiple of 16, every
// pointer 16-B aligned.
#include "lfa_kernels.hpp"


namespace {
template <bool UW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void tp_probe_w2(
    lfa::PutArgs a, size_t nvec) {
  lfa::tree_put_body<lfa::OP_SUM, int8_t, 16, 4, UW>(a, nvec);
}
}  // namespace

extern "C" int lfa__tp_probe(int form, void *const *dsts, int ndst, const void *const *srcs,
                             int nsrc, size_t cnt, void *stream) {
  using namespace lfa;
  if (nsrc < 16 || nsrc > 31 || ndst < 1 || ndst > kMaxPut || cnt % 16) return -LFA_EINVAL;
  PutArgs a;
  tree_leaves(a.t, srcs, nsrc);
  memset(a.out, 0, sizeof(a.out));
  a.nout = ndst;
  for (int j = 0; j < ndst; j++) a.out[j] = dsts[j];
  const size_t nvec = cnt / 16;
  const dim3 grid(grid_for(nvec, (size_t)kBlock * 4, 0x7fffffffu));
  if (form == 0)
    hipLaunchKernelGGL((reduce_tree_put<OP_SUM, int8_t, 16, 4, false>), grid, dim3(kBlock), 0,
                       (hipStream_t)stream, a, nvec);
  else if (form == 1)
    hipLaunchKernelGGL((reduce_tree_put<OP_SUM, int8_t, 16, 4, true>), grid, dim3(kBlock), 0,
                       (hipStream_t)stream, a, nvec);
  else if (form == 2)
    hipLaunchKernelGGL((tp_probe_w2<true>), grid, dim3(kBlock), 0, (hipStream_t)stream, a, nvec);
  else if (form == 3)
    hipLaunchKernelGGL((tp_probe_w2<false>), grid, dim3(kBlock), 0, (hipStream_t)stream, a, nvec);
  else
    return -LFA_EINVAL;
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}
