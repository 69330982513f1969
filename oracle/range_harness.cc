// ORACLE TEST INFRASTRUCTURE -- the reference's UNMODIFIED src/util/range.h
// (Range<T>::EvenDivide, Project, SetIntersection), compiled with a PbRange
// stand-in (ref_stub_range/) and throwing CHECKs.  Built by `make -C oracle
// ref` into oracle/_ref/libpsrange.so.
#include <stdint.h>
#include <algorithm>
#include <sstream>
#include <stdexcept>
#include <string>

namespace range_check {
struct Fail {
  std::ostringstream ss;
  ~Fail() noexcept(false) { throw std::runtime_error(ss.str()); }
};
}  // namespace range_check
#define CHECK(c) if (c) ; else range_check::Fail().ss
#define CHECK_GT(a, b) CHECK((a) > (b))
#define CHECK_LT(a, b) CHECK((a) < (b))

#include "util/range.h"

extern "C" int psref_even_divide(uint64_t begin, uint64_t end, uint64_t n, uint64_t i,
                                 uint64_t* ob, uint64_t* oe) {
  try {
    PS::Range<uint64_t> r(begin, end);
    auto d = r.EvenDivide(n, i);
    *ob = d.begin();
    *oe = d.end();
    return 0;
  } catch (const std::exception&) {
    return -1;
  }
}

extern "C" uint64_t psref_project(uint64_t begin, uint64_t end, uint64_t v) {
  return PS::Range<uint64_t>(begin, end).Project(v);
}
