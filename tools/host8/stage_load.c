/* One emulated rank's host-side staging load: at 8 ranks per node each rank's
 * pageable H2D copies make the HIP runtime memcpy its ~1.06 GB signature stream (and tables) into
 * pinned bounce buffers every ~36-ms step, on the rank's own 2 host threads. This program does the
 * same memory work with no GPU at all: `threads` threads each memcpy their share of a `mb`-MB source
 * into a destination ring, paced to `gbps` GB/s for the whole process, for `seconds`. Run 7 of them
 * beside one real rank (tools/host8/run.sh) to see what the other ranks' staging does to it.
 * With a 5th argument "read" the threads only read the source (a registered rank's DMA engines read
 * its pages without any CPU copy: the other ranks' host-memory traffic then, minus the staging writes).
 * usage: stage_load <threads> <MB per step> <step ms> <seconds> [read] */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

typedef struct {
  uint8_t *src, *dst;
  size_t bytes;
  double step_s, until;
  double copied;
  int read_only;
  uint64_t sink;
} job;

static void* run(void* p) {
  job* j = (job*)p;
  const size_t piece = 4u << 20; /* the runtime stages in MB-sized pieces */
  double t0 = now();
  uint64_t steps = 0;
  while (now() < j->until) {
    for (size_t o = 0; o < j->bytes; o += piece) {
      const size_t n = j->bytes - o < piece ? j->bytes - o : piece;
      if (j->read_only) {
        const uint64_t* q = (const uint64_t*)(j->src + o);
        uint64_t x = 0;
        for (size_t k = 0; k < n / 8; k += 8) x += q[k] ^ q[k + 1] ^ q[k + 2] ^ q[k + 3] ^ q[k + 4] ^ q[k + 5] ^ q[k + 6] ^ q[k + 7];
        j->sink += x;
      } else {
        memcpy(j->dst + (o % (64u << 20)), j->src + o, n);
      }
    }
    j->copied += (double)j->bytes;
    ++steps;
    const double next = t0 + steps * j->step_s; /* pace: one step's bytes per step period */
    double t = now();
    if (t < next) {
      struct timespec ts = {(time_t)(next - t), (long)((next - t - (time_t)(next - t)) * 1e9)};
      nanosleep(&ts, NULL);
    }
  }
  return NULL;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s threads MB_per_step step_ms seconds [read]\n", argv[0]);
    return 2;
  }
  const int nt = atoi(argv[1]);
  const size_t bytes = (size_t)atol(argv[2]) << 20;
  const double step_s = atof(argv[3]) / 1e3, secs = atof(argv[4]);
  job* jobs = calloc(nt, sizeof(job));
  pthread_t* th = calloc(nt, sizeof(pthread_t));
  const double until = now() + secs;
  for (int t = 0; t < nt; ++t) {
    jobs[t].bytes = bytes / nt;
    jobs[t].src = malloc(jobs[t].bytes);
    jobs[t].dst = malloc(64u << 20);
    memset(jobs[t].src, t + 1, jobs[t].bytes);
    memset(jobs[t].dst, 0, 64u << 20);
    jobs[t].step_s = step_s;
    jobs[t].until = until;
    jobs[t].read_only = argc > 5 && strcmp(argv[5], "read") == 0;
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  double tot = 0;
  uint64_t sink = 0;
  for (int t = 0; t < nt; ++t) {
    pthread_join(th[t], NULL);
    tot += jobs[t].copied;
    sink += jobs[t].sink;
  }
  printf("{\"threads\": %d, \"GBps\": %.2f, \"mode\": \"%s\", \"sink\": %llu}\n", nt, tot / secs / 1e9,
         jobs[0].read_only ? "read" : "copy", (unsigned long long)(sink & 1));
  return 0;
}
