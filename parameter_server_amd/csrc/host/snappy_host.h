// COMPRESSING buffers: compress / uncompress several arrays of a message with
// one wait at the end (each kernel chain publishes its stream length / verdict
// to its own host-mapped slot).
#pragma once
#include <vector>

#include "context.h"

namespace psf {

uint32_t snappy_parse_header(const uint8_t* p, size_t n, uint64_t* len);
// header of a (device or host) buffer; 0 when malformed
uint32_t snappy_read_header(Context& c, const Buffer& in, uint64_t* len);

class SnappyBatch {
 public:
  explicit SnappyBatch(Context& c) : c_(c) {}
  // *dst is assigned at flush(); src must stay alive until then
  void compress(const Buffer& src, Buffer* dst);
  void uncompress(const Buffer& src, Buffer* dst);
  void flush();

 private:
  struct Job {
    Buffer in, out;
    Buffer* dst = nullptr;
    int slot = 0;
    uint32_t ticket = 0;
  };
  Context& c_;
  std::vector<Job> jobs_;
};

}  // namespace psf
