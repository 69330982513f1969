// Native exchange of the cross-range spill (see exchange.h).
#include "exchange.h"

#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/statvfs.h>
#include <time.h>
#include <unistd.h>

#include <rccl/rccl.h>

namespace psf {

// ------------------------------------------------------------- librccl ----
// Loaded on first use (a process that never spills needs no RCCL; in a
// PyTorch process the soname resolves to the librccl torch already loaded).
namespace {
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  static std::string err;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      err = std::string("librccl not found: ") + dlerror();
      return;
    }
    auto sym = [&](const char* n) {
      void* p = dlsym(h, n);
      if (!p && err.empty()) err = std::string("librccl lacks ") + n;
      return p;
    };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.init_rank = reinterpret_cast<decltype(r.init_rank)>(sym("ncclCommInitRank"));
    r.destroy = reinterpret_cast<decltype(r.destroy)>(sym("ncclCommDestroy"));
    r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
    r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
  });
  if (!err.empty()) throw CheckError(kErrUnsupported, err);
  return r;
}

void nccl_check(ncclResult_t e, const char* what) {
  if (e != ncclSuccess)
    throw CheckError(kErrHip, std::string(what) + ": " + (rccl().error_string ? rccl().error_string(e) : "?"));
}

constexpr uint32_t kMagic = 0x50534558u;  // 'PSEX'
constexpr int kMaxWorld = 64;
constexpr uint64_t kPage = 4096;
constexpr uint64_t up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }
}  // namespace

void rccl_unique_id(void* out128) {
  ncclUniqueId id;
  nccl_check(rccl().get_unique_id(&id), "ncclGetUniqueId");
  memcpy(out128, &id, sizeof(id));
}

// --------------------------------------------------------------- layout ----
struct Exchange::Shared {
  std::atomic<uint32_t> magic;
  uint32_t world;
  uint64_t meta_cap, host_cap, box_bytes;
  std::atomic<uint32_t> attached;
  std::atomic<uint32_t> failed;  // 0, or 1 + the first rank whose step failed (Exchange::fail)
  uint8_t pad0[128 - 40];
  struct Ctl {
    std::atomic<uint64_t> posted;    // steps this rank has posted
    std::atomic<uint64_t> consumed;  // steps this rank has read from every source
    uint8_t pad[112];
  } ctl[kMaxWorld];
};
static_assert(sizeof(std::atomic<uint64_t>) == 8, "lock-free 64-bit atomics");
constexpr uint64_t kHeader = up(sizeof(Exchange::Shared), kPage);

// one bank of one rank: per destination the record / data byte counts and
// offsets, then the records area (meta_cap), then the data area (host_cap)
struct Exchange::RankBox {
  int64_t meta[kMaxWorld];
  int64_t pay[kMaxWorld];
  uint64_t rec_off[kMaxWorld];
  uint64_t pay_off[kMaxWorld];
  uint8_t* records() { return reinterpret_cast<uint8_t*>(this) + kPage; }
};
static_assert(sizeof(Exchange::RankBox) <= kPage, "box header");

Exchange::RankBox* Exchange::box(int r, int bank) const {
  return reinterpret_cast<RankBox*>(base_ + kHeader + ((uint64_t)r * 2 + bank) * box_bytes_);
}

namespace {
std::atomic<bool> g_self_p2p{false};
}
void set_exchange_self_p2p(bool on) { g_self_p2p.store(on, std::memory_order_relaxed); }

void Exchange::unref(Exchange* e) {
  if (!e || e->refs.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
  Context* c = e->ctx_;
  delete e;
  Context::unref(c);
}

void Exchange::check_failed() const {
  if (!failed_.empty()) throw CheckError(kErrCheck, "exchange: an earlier step failed on this rank: " + failed_);
  const uint32_t f = sh_ ? sh_->failed.load(std::memory_order_acquire) : 0;
  if (f) throw CheckError(kErrCheck, "exchange: rank " + std::to_string(f - 1) + " failed a step");
}

void Exchange::fail(const std::string& why) {
  if (failed_.empty()) failed_ = why.empty() ? "unknown error" : why;
  uint32_t none = 0;
  if (sh_) sh_->failed.compare_exchange_strong(none, (uint32_t)rank_ + 1, std::memory_order_acq_rel);
  gathered_ = false;
}

void Exchange::wait_until(const std::atomic<uint64_t>* v, uint64_t want, const char* what, int who) {
  if (v->load(std::memory_order_acquire) >= want) return;
  const int64_t t0 = now_ns();
  for (uint64_t spin = 0;; ++spin) {
    if (v->load(std::memory_order_acquire) >= want) break;
    if ((spin & 255) == 0) check_failed();
    if (spin > 2048) {
      sched_yield();
      if ((spin & 1023) == 0 && (double)(now_ns() - t0) * 1e-9 > timeout_s_)
        throw CheckError(kErrHip, std::string("exchange: rank ") + std::to_string(who) + " did not " + what +
                                      " step " + std::to_string(want - 1) + " within " +
                                      std::to_string((int)timeout_s_) + " s");
    }
  }
  wait_ns += now_ns() - t0;
}

Exchange::Exchange(Context* ctx, int rank, int world, const std::string& path, Transport t, const void* nccl_id,
                   uint64_t meta_cap, uint64_t host_cap)
    : ctx_(ctx), rank_(rank), world_(world), transport_(t), path_(path) {
  if (world <= 0 || world > kMaxWorld || rank < 0 || rank >= world)
    throw CheckError(kErrArg, "exchange: bad rank / world (at most 64 ranks)");
  if (t == kRccl && ctx->device() < 0) throw CheckError(kErrArg, "exchange: RCCL needs a device context");
  if (t == kRccl && !nccl_id) throw CheckError(kErrArg, "exchange: RCCL needs the unique id");
  if (path.empty() || path.find('/') != std::string::npos)
    throw CheckError(kErrArg, "exchange: the mailbox name is a file name");
  if (const char* e = getenv("PSF_EXCHANGE_TIMEOUT_S")) {
    const double v = atof(e);
    if (v > 0) timeout_s_ = v;
  }
  meta_cap_ = up(meta_cap ? meta_cap : (1u << 20), kPage);
  host_cap_ = t == kHost ? up(host_cap ? host_cap : (64u << 20), kPage) : 0;
  box_bytes_ = kPage + meta_cap_ + host_cap_;
  map_bytes_ = kHeader + (uint64_t)world * 2 * box_bytes_;
  meta_in_.assign(world, 0);
  pay_in_.assign(world, 0);

  // the mailbox file: /dev/shm when it has room, else the temp directory
  // (PSF_EXCHANGE_DIR overrides); rank 0 creates it, the others look in both
  std::vector<std::string> dirs;
  if (const char* e = getenv("PSF_EXCHANGE_DIR")) dirs.push_back(e);
  dirs.push_back("/dev/shm");
  const char* tmp = getenv("TMPDIR");
  dirs.push_back(tmp && *tmp ? tmp : "/tmp");
  int fd = -1;
  const int64_t t0 = now_ns();
  if (rank == 0) {
    std::string err;
    for (const std::string& d : dirs) {
      struct statvfs sv;
      if (statvfs(d.c_str(), &sv) != 0 || (uint64_t)sv.f_bavail * sv.f_frsize < map_bytes_ + (16u << 20)) continue;
      const std::string p = d + "/" + path;
      fd = open(p.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) {
        err = p + ": " + strerror(errno);
        continue;
      }
      if (ftruncate(fd, (off_t)map_bytes_) != 0) {
        err = p + ": ftruncate: " + strerror(errno);
        close(fd);
        unlink(p.c_str());
        fd = -1;
        continue;
      }
      path_ = p;
      break;
    }
    if (fd < 0) throw CheckError(kErrHip, "exchange: cannot create the mailbox " + (err.empty() ? path : err));
  } else {
    for (;;) {
      for (const std::string& d : dirs) {
        const std::string p = d + "/" + path;
        fd = open(p.c_str(), O_RDWR);
        if (fd < 0) continue;
        struct stat st;
        if (fstat(fd, &st) == 0 && (uint64_t)st.st_size == map_bytes_) {
          path_ = p;
          break;
        }
        close(fd);
        fd = -1;
      }
      if (fd >= 0) break;
      if ((double)(now_ns() - t0) * 1e-9 > timeout_s_) throw CheckError(kErrHip, "exchange: no mailbox " + path);
      usleep(1000);
    }
  }
  void* m = mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) throw CheckError(kErrHip, std::string("exchange: mmap: ") + strerror(errno));
  base_ = static_cast<uint8_t*>(m);
  sh_ = reinterpret_cast<Shared*>(base_);
  if (rank == 0) {
    sh_->world = (uint32_t)world;
    sh_->meta_cap = meta_cap_;
    sh_->host_cap = host_cap_;
    sh_->box_bytes = box_bytes_;
    sh_->magic.store(kMagic, std::memory_order_release);
  } else {
    while (sh_->magic.load(std::memory_order_acquire) != kMagic) {
      if ((double)(now_ns() - t0) * 1e-9 > timeout_s_) throw CheckError(kErrHip, "exchange: mailbox never initialised");
      usleep(100);
    }
    if (sh_->world != (uint32_t)world || sh_->box_bytes != box_bytes_)
      throw CheckError(kErrArg, "exchange: ranks disagree on world / capacities");
  }
  sh_->attached.fetch_add(1, std::memory_order_acq_rel);
  while (sh_->attached.load(std::memory_order_acquire) < (uint32_t)world) {
    if ((double)(now_ns() - t0) * 1e-9 > timeout_s_) throw CheckError(kErrHip, "exchange: not every rank attached");
    usleep(100);
  }
  if (rank == 0) unlink(path_.c_str());  // mapped by every rank: the name is no longer needed

  if (t == kRccl) {
    DeviceScope ds(ctx->device());
    ncclUniqueId id;
    memcpy(&id, nccl_id, sizeof(id));
    ncclComm_t c = nullptr;
    nccl_check(rccl().init_rank(&c, world, id, rank), "ncclCommInitRank");
    comm_ = c;
    PSF_HIP_CHECK(hipStreamCreateWithFlags(&cstream_, hipStreamNonBlocking));
    PSF_HIP_CHECK(hipEventCreateWithFlags(&ev_sent_, hipEventDisableTiming));
    PSF_HIP_CHECK(hipEventCreateWithFlags(&ev_done_, hipEventDisableTiming));
  }
}

Exchange::~Exchange() {
  if (comm_ || cstream_) {
    DeviceScope ds(ctx_->device(), true);
    if (cstream_) (void)hipStreamSynchronize(cstream_);
    if (comm_) (void)rccl().destroy(static_cast<ncclComm_t>(comm_));
    if (cstream_) (void)hipStreamDestroy(cstream_);
    if (ev_sent_) (void)hipEventDestroy(ev_sent_);
    if (ev_done_) (void)hipEventDestroy(ev_done_);
  }
  if (base_) munmap(base_, map_bytes_);
}

void Exchange::post(const int64_t* meta, const int64_t* pay, const uint8_t* const* records, const uint8_t* send,
                    const uint64_t* soff) {
  check_failed();
  if (gathered_) throw CheckError(kErrArg, "exchange: post() before the last step's move()");
  const uint64_t k = step_;
  const int bank = (int)(k & 1);
  // bank k & 1 was last read in step k - 2: every rank must be done with it
  if (k >= 2)
    for (int r = 0; r < world_; ++r) wait_until(&sh_->ctl[r].consumed, k - 1, "consume", r);
  RankBox* b = box(rank_, bank);
  uint64_t ro = 0, po = 0;
  for (int d = 0; d < world_; ++d) {
    if (meta[d] < 0 || pay[d] < 0) throw CheckError(kErrArg, "exchange: negative size");
    b->meta[d] = meta[d];
    b->pay[d] = pay[d];
    b->rec_off[d] = ro;
    b->pay_off[d] = po;
    ro += (uint64_t)meta[d];
    po += (uint64_t)pay[d];
    if (d != rank_) bytes_sent += meta[d] + pay[d];
  }
  if (ro > meta_cap_)
    throw CheckError(kErrArg, "exchange: Task records of one step exceed the mailbox (" + std::to_string(ro) +
                                  " > " + std::to_string(meta_cap_) + " bytes)");
  if (transport_ == kHost && po > host_cap_)
    throw CheckError(kErrArg, "exchange: data of one step exceed the host mailbox (" + std::to_string(po) +
                                  " > " + std::to_string(host_cap_) + " bytes)");
  for (int d = 0; d < world_; ++d)
    if (meta[d]) memcpy(b->records() + b->rec_off[d], records[d], (size_t)meta[d]);
  if (transport_ == kHost && po) {
    uint8_t* h = b->records() + meta_cap_;
    if (ctx_->device() >= 0) {
      ctx_->sync();  // the gather that filled `send` is done
      for (int d = 0; d < world_; ++d)
        if (pay[d]) PSF_HIP_CHECK(hipMemcpy(h + b->pay_off[d], send + soff[d], (size_t)pay[d], hipMemcpyDeviceToHost));
    } else {
      for (int d = 0; d < world_; ++d)
        if (pay[d]) memcpy(h + b->pay_off[d], send + soff[d], (size_t)pay[d]);
    }
  }
  sh_->ctl[rank_].posted.store(k + 1, std::memory_order_release);
  step_ = k + 1;
  ++steps;
}

void Exchange::gather_meta() {
  check_failed();
  if (gathered_) return;
  const uint64_t k = step_ - 1;
  if (step_ == 0) throw CheckError(kErrArg, "exchange: gather before post");
  for (int s = 0; s < world_; ++s) {
    wait_until(&sh_->ctl[s].posted, k + 1, "post", s);
    const RankBox* b = box(s, (int)(k & 1));
    meta_in_[s] = b->meta[rank_];
    pay_in_[s] = b->pay[rank_];
  }
  gathered_ = true;
}

const uint8_t* Exchange::records_in(int s) const {
  const uint64_t k = step_ - 1;
  RankBox* b = box(s, (int)(k & 1));
  return b->records() + b->rec_off[rank_];
}

void Exchange::move(const uint8_t* send, const uint64_t* soff, uint8_t* recv, const uint64_t* roff) {
  check_failed();
  if (!gathered_) gather_meta();
  const uint64_t k = step_ - 1;
  const int bank = (int)(k & 1);
  if (transport_ == kHost) {
    for (int s = 0; s < world_; ++s) {
      if (!pay_in_[s]) continue;
      RankBox* b = box(s, bank);
      const uint8_t* h = b->records() + meta_cap_ + b->pay_off[rank_];
      copied_bytes += pay_in_[s];
      if (ctx_->device() >= 0)
        PSF_HIP_CHECK(hipMemcpyAsync(recv + roff[s], h, (size_t)pay_in_[s], hipMemcpyHostToDevice, ctx_->stream()));
      else
        memcpy(recv + roff[s], h, (size_t)pay_in_[s]);
    }
    // (pageable sources: the copies are done with the mailbox when the
    // stream has passed them)
    if (ctx_->device() >= 0) ctx_->sync();
  } else {
    const RankBox* mine = box(rank_, bank);
    hipStream_t st = ctx_->stream();
    PSF_HIP_CHECK(hipEventRecord(ev_sent_, st));  // the send buffer is filled
    PSF_HIP_CHECK(hipStreamWaitEvent(cstream_, ev_sent_, 0));
    // the self slice: a device copy, or (test knob) a send / recv to self in
    // the group like every other peer's
    const bool self_p2p = g_self_p2p.load(std::memory_order_relaxed);
    if (pay_in_[rank_] && !self_p2p) {
      PSF_HIP_CHECK(hipMemcpyAsync(recv + roff[rank_], send + soff[rank_], (size_t)pay_in_[rank_],
                                   hipMemcpyDeviceToDevice, cstream_));
      copied_bytes += pay_in_[rank_];
    }
    const Rccl& R = rccl();
    ncclComm_t c = static_cast<ncclComm_t>(comm_);
    nccl_check(R.group_start(), "ncclGroupStart");
    for (int p = 0; p < world_; ++p) {
      if (p == rank_ && !self_p2p) continue;
      if (mine->pay[p]) {
        nccl_check(R.send(send + soff[p], (size_t)mine->pay[p], ncclUint8, p, c, cstream_), "ncclSend");
        rccl_bytes += mine->pay[p];
        ++rccl_sends;
      }
      if (pay_in_[p]) nccl_check(R.recv(recv + roff[p], (size_t)pay_in_[p], ncclUint8, p, c, cstream_), "ncclRecv");
    }
    nccl_check(R.group_end(), "ncclGroupEnd");
    PSF_HIP_CHECK(hipEventRecord(ev_done_, cstream_));
    // the context's stream goes on with other work and waits for the data
    // only where the caller joins (join_data)
  }
  sh_->ctl[rank_].consumed.store(k + 1, std::memory_order_release);
  gathered_ = false;
}

void Exchange::join_data() {
  if (transport_ == kRccl) PSF_HIP_CHECK(hipStreamWaitEvent(ctx_->stream(), ev_done_, 0));
}

}  // namespace psf
