// CPU emulation driver for hsds_amd/csrc/region.h (TEST INFRASTRUCTURE ONLY): every lane
// of every wave of copy_kernel / compare_kernel in turn, over host buffers, so the copy and
// compare paths (run slots at every relative alignment, gathers, element fallbacks, row
// grouping) are checked against a numpy model on CPU.  Never used by the product.
#include "../../hsds_amd/csrc/region.h"

extern "C" int emu_copy(const uint8_t* src, uint8_t* dst, const hsds_copy_desc* descs, int64_t n, const int32_t* flags,
                        uint32_t nwaves) {
  for (int64_t di = 0; di < n; di++) {
    if (flags && !flags[di]) continue;
    rg::NReg r;
    if (!rg::nreg_make(descs[di], 1, r)) continue;
    const rg::Plan p = rg::plan_copy(r);
    for (uint32_t w = 0; w < nwaves; w++)
      for (uint64_t g = w; g < p.ngroups; g += nwaves)
        for (uint32_t lane = 0; lane < 64; lane++) rg::copy_group(src, dst, r, p, g, lane);
  }
  return 0;
}

extern "C" int emu_compare(const uint8_t* b, const uint8_t* a, const hsds_copy_desc* descs, int64_t n, int kind,
                           int32_t* differs) {
  for (int64_t di = 0; di < n; di++) {
    differs[di] = 0;
    rg::NReg r;
    if (!rg::nreg_make(descs[di], kind == HSDS_KIND_BYTES, r)) continue;
    const rg::Plan p = rg::plan_compare(r);
    for (uint64_t g = 0; g < p.ngroups && !differs[di]; g++)
      for (uint32_t lane = 0; lane < 64; lane++)
        if (rg::compare_group(b, a, r, p, g, lane, kind)) differs[di] = 1;
  }
  return 0;
}
