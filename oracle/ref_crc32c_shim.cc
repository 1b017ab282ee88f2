// TEST INFRASTRUCTURE ONLY.  C entry points onto the reference's own
// crc32c::Extend (reference src/util/crc32c.cc:283) and Mask/Unmask
// (src/util/crc32c.h:29-38), compiled in place from /root/reference by
// oracle/Makefile into oracle/_ref/.  Used by tests to pin
// oracle/psg_oracle.c's restatement and the GPU kernel.
#include "util/crc32c.h"
extern "C" unsigned ref_crc32c_extend(unsigned init, const char* data, size_t n) {
  return PS::crc32c::Extend(init, data, n);
}
extern "C" unsigned ref_crc32c_mask(unsigned crc) { return PS::crc32c::Mask(crc); }
extern "C" unsigned ref_crc32c_unmask(unsigned crc) { return PS::crc32c::Unmask(crc); }
