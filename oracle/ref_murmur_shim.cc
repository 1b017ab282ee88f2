// TEST INFRASTRUCTURE ONLY.  C entry point onto the reference's own
// MurmurHash3_x64_128 (reference src/util/MurmurHash3.cc:255), compiled in
// place from /root/reference by oracle/Makefile into oracle/_ref/.  Used by
// tests to pin oracle/psg_oracle.c's restatement of the CTR key shuffle.
#include "util/MurmurHash3.h"
extern "C" void ref_murmur3_x64_128(const void* key, int len, unsigned seed,
                                    void* out) {
  MurmurHash3_x64_128(key, len, seed, out);
}
