// Diagnostic: a sampling profiler for the host side of a run (no perf on the
// GPU box).  sampler_start(us) arms a POSIX CLOCK_MONOTONIC timer aimed at
// the calling thread (ITIMER_PROF only ticks at the scheduler's rate, a few
// ms); each SIGPROF records up to 8 return addresses (backtrace(), primed
// before arming).  Wall-clock sampling: blocked time is sampled too.  sampler_stop(path) disarms and writes
// the samples plus /proc/self/maps to `path`; tools/sampler_report.py
// resolves them against the built libraries.  Build:
//   gcc -O2 -shared -fPIC -o tools/libsampler.so tools/sampler.c -lrt
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdio.h>
#include <string.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#define MAXS 200000
#define DEPTH 8
static void* g_frames[MAXS][DEPTH];
static unsigned char g_depth[MAXS];
static atomic_int g_n;
static pid_t g_tid;
static atomic_int g_other;
static timer_t g_timer;

static void on_prof(int sig, siginfo_t* si, void* uc) {
  (void)sig;
  (void)si;
  (void)uc;
  if ((pid_t)syscall(SYS_gettid) != g_tid) {
    atomic_fetch_add(&g_other, 1);
    return;
  }
  const int i = atomic_fetch_add(&g_n, 1);
  if (i >= MAXS) return;
  g_depth[i] = (unsigned char)backtrace(g_frames[i], DEPTH);
}

int sampler_start(int period_us) {
  void* prime[4];
  backtrace(prime, 4);  // loads libgcc's unwinder outside the handler
  g_tid = (pid_t)syscall(SYS_gettid);
  atomic_store(&g_n, 0);
  atomic_store(&g_other, 0);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, NULL)) return -1;
  struct sigevent ev;
  memset(&ev, 0, sizeof ev);
  ev.sigev_notify = SIGEV_THREAD_ID;
  ev.sigev_signo = SIGPROF;
  ev._sigev_un._tid = g_tid;
  if (timer_create(CLOCK_MONOTONIC, &ev, &g_timer)) return -2;
  struct itimerspec it;
  it.it_interval.tv_sec = 0;
  it.it_interval.tv_nsec = (long)period_us * 1000;
  it.it_value = it.it_interval;
  return timer_settime(g_timer, 0, &it, NULL);
}

int sampler_stop(const char* path) {
  timer_delete(g_timer);
  signal(SIGPROF, SIG_IGN);
  FILE* f = fopen(path, "w");
  if (!f) return -1;
  int n = atomic_load(&g_n);
  if (n > MAXS) n = MAXS;
  fprintf(f, "# samples %d other_threads %d\n", n, atomic_load(&g_other));
  for (int i = 0; i < n; ++i) {
    fprintf(f, "S");
    for (int d = 0; d < g_depth[i]; ++d) fprintf(f, " %lx", (unsigned long)g_frames[i][d]);
    fprintf(f, "\n");
  }
  FILE* m = fopen("/proc/self/maps", "r");
  if (m) {
    char line[1024];
    while (fgets(line, sizeof line, m)) fprintf(f, "M %s", line);
    fclose(m);
  }
  fclose(f);
  return n;
}
