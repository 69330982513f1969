// ORACLE TEST INFRASTRUCTURE: stand-in for the protoc-generated PbRange
// (src/util/proto/range.proto: required uint64 begin = 1, end = 2) so the
// reference's unmodified src/util/range.h compiles here.
#pragma once
#include <stdint.h>
namespace PS {
class PbRange {
 public:
  uint64_t begin() const { return b_; }
  uint64_t end() const { return e_; }
  void set_begin(uint64_t v) { b_ = v; }
  void set_end(uint64_t v) { e_ = v; }
 private:
  uint64_t b_ = 0, e_ = 0;
};
}  // namespace PS
