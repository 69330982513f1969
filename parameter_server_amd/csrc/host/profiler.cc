// Launch profiler: a start/stop hipEvent pair recorded on the launch stream
// around each kernel (the bench's live per-kernel durations, cross-checked
// against rocprofv3 --kernel-trace in profiles/).
#include <stdlib.h>

#include "../psf_internal.h"

namespace psf {

Profiler::~Profiler() {
  for (int i = 0; i < npend_; ++i) {
    (void)hipEventDestroy(pend_[i].a);
    (void)hipEventDestroy(pend_[i].b);
  }
  for (int i = 0; i < npool_; ++i) (void)hipEventDestroy(pool_[i]);
  free(pend_);
  free(pool_);
}

hipEvent_t Profiler::take() {
  if (npool_ > 0) return pool_[--npool_];
  hipEvent_t e = nullptr;
  // timing only: no system-scope fence at record (it wrote back and
  // invalidated the caches inside the timed bracket: +1.5 us per encode
  // launch, +4 us per C2 step, measured A/B on one box)
  (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  return e;
}

void Profiler::pool_push(hipEvent_t e) {
  if (npool_ + 1 > cappool_) {
    cappool_ = cappool_ ? 2 * cappool_ : 128;
    pool_ = static_cast<hipEvent_t*>(realloc(pool_, sizeof(hipEvent_t) * cappool_));
  }
  pool_[npool_++] = e;
}

void Profiler::begin(hipStream_t st) {
  cur_ = take();
  (void)hipEventRecord(cur_, st);
}

thread_local ExtEvents g_ext_events;

void Profiler::begin_ext() {
  cur_ = take();
  cur_b_ = take();
  g_ext_events = ExtEvents{cur_, cur_b_};
}

void Profiler::end(KernelId id, hipStream_t st, double alg_bytes) {
  hipEvent_t b;
  if (cur_b_) {
    b = cur_b_;
    cur_b_ = nullptr;
    if (g_ext_events.a == cur_) {  // the scope launched nothing through psf_launch
      g_ext_events = ExtEvents{};
      pool_push(cur_);
      pool_push(b);
      cur_ = nullptr;
      return;
    }
  } else {
    b = take();
    (void)hipEventRecord(b, st);
  }
  if (npend_ == cap_) {
    cap_ = cap_ ? 2 * cap_ : 64;
    pend_ = static_cast<Pending*>(realloc(pend_, sizeof(Pending) * cap_));
  }
  pend_[npend_++] = Pending{id, cur_, b, alg_bytes};
  cur_ = nullptr;
  if (npend_ >= 4096) collect();
}

void Profiler::collect() {
  for (int i = 0; i < npend_; ++i) {
    Pending& p = pend_[i];
    float ms = 0.f;
    (void)hipEventSynchronize(p.b);
    (void)hipEventElapsedTime(&ms, p.a, p.b);
    launches[p.id] += 1;
    total_ms[p.id] += ms;
    bytes[p.id] += p.bytes;
    pool_push(p.a);
    pool_push(p.b);
  }
  npend_ = 0;
}

void Profiler::reset() {
  collect();
  for (int k = 0; k < kKNum; ++k) { launches[k] = 0; total_ms[k] = 0; bytes[k] = 0; }
}

}  // namespace psf
