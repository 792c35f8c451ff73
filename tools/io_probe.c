// Host file I/O rates on the box (for the file -> file entry point's design): pread of
// a page-cached file and writes of a new file, with 1..16 threads; unlink time.
//   gcc -O2 -pthread tools/io_probe.c -o /tmp/io_probe && /tmp/io_probe DIR
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

static double now(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + t.tv_nsec * 1e-9; }
typedef struct { int fd; uint8_t* buf; uint64_t off, len; int mode; } Job;
static void* run(void* a) {
  Job* j = (Job*)a;
  uint64_t done = 0;
  while (done < j->len) {
    size_t n = j->len - done > (4u << 20) ? (4u << 20) : j->len - done;
    ssize_t r = j->mode == 0 ? pread(j->fd, j->buf + done, n, j->off + done) : pwrite(j->fd, j->buf + done, n, j->off + done);
    if (r <= 0) break;
    done += r;
  }
  return NULL;
}
static double par(int fd, uint8_t* buf, uint64_t len, int nt, int mode) {
  pthread_t th[64]; Job jobs[64];
  double t0 = now();
  for (int i = 0; i < nt; i++) {
    uint64_t a = len * i / nt, b = len * (i + 1) / nt;
    jobs[i] = (Job){fd, buf + a, a, b - a, mode};
    pthread_create(&th[i], NULL, run, &jobs[i]);
  }
  for (int i = 0; i < nt; i++) pthread_join(th[i], NULL);
  return now() - t0;
}
typedef struct { uint8_t* dst; const uint8_t* src; uint64_t len; } Cp;
static void* cp(void* a) { Cp* c = (Cp*)a; memcpy(c->dst, c->src, c->len); return NULL; }
int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp";
  char lp[512], sp[512];
  snprintf(lp, sizeof lp, "%s/io_probe.log", dir);
  snprintf(sp, sizeof sp, "%s/io_probe.spi", dir);
  const uint64_t L = 1180000084ull, S = 208000128ull;
  uint8_t* buf = aligned_alloc(4096, L);
  memset(buf, 7, L);
  int fd = open(lp, O_RDWR | O_CREAT | O_TRUNC, 0644);
  double t = par(fd, buf, L, 8, 1);
  printf("write 1.18 GB log (8 thr): %.1f ms\n", t * 1e3);
  for (int nt = 1; nt <= 32; nt *= 2) {
    t = par(fd, buf, L, nt, 0);
    printf("pread 1.18 GB cached, %2d threads: %.1f ms = %.1f GB/s\n", nt, t * 1e3, L / t / 1e9);
  }
  close(fd);
  for (int nt = 1; nt <= 32; nt *= 2) {
    unlink(sp);
    int o = open(sp, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    t = par(o, buf, S, nt, 1);
    double t2 = now();
    close(o);
    double t3 = now();
    unlink(sp);
    printf("pwrite 208 MB new file, %2d threads: %.1f ms = %.1f GB/s (close %.1f ms, unlink %.1f ms)\n", nt, t * 1e3,
           S / t / 1e9, (t3 - t2) * 1e3, (now() - t3) * 1e3);
  }
  for (int nt = 1; nt <= 32; nt *= 2) {
    int o = open(sp, O_RDWR | O_CREAT | O_TRUNC, 0644);
    double t0 = now();
    if (ftruncate(o, S)) return 1;
    uint8_t* m = mmap(NULL, S, PROT_READ | PROT_WRITE, MAP_SHARED, o, 0);
    pthread_t th[64]; Cp c[64];
    for (int i = 0; i < nt; i++) {
      uint64_t a = S * i / nt, b = S * (i + 1) / nt;
      c[i] = (Cp){m + a, buf + a, b - a};
      pthread_create(&th[i], NULL, cp, &c[i]);
    }
    for (int i = 0; i < nt; i++) pthread_join(th[i], NULL);
    munmap(m, S);
    close(o);
    t = now() - t0;
    unlink(sp);
    printf("mmap write 208 MB new file, %2d threads: %.1f ms = %.1f GB/s\n", nt, t * 1e3, S / t / 1e9);
  }
  // O_DIRECT (page cache bypassed: no inode-lock serialisation of buffered writes), 4 KiB-aligned
  // pieces from 1..32 threads, into a new file and into one preallocated with fallocate
  for (int pre = 0; pre < 2; pre++)
    for (int nt = 1; nt <= 32; nt *= 2) {
      unlink(sp);
      int o = open(sp, O_WRONLY | O_CREAT | O_TRUNC | O_DIRECT, 0644);
      if (o < 0) {
        printf("O_DIRECT open failed: %s\n", strerror(errno));
        break;
      }
      double t0 = now();
      if (pre && fallocate(o, 0, 0, S) != 0) printf("fallocate failed: %s\n", strerror(errno));
      const uint64_t SA = (S + 4095) & ~4095ull;
      t = par(o, buf, SA, nt, 1);
      double t2 = now();
      if (ftruncate(o, S)) return 1;
      close(o);
      printf("O_DIRECT pwrite 208 MB%s, %2d threads: %.1f ms = %.1f GB/s (all %.1f ms)\n", pre ? " (fallocated)" : "",
             nt, t * 1e3, S / t / 1e9, (now() - t0) * 1e3);
      (void)t2;
    }
  unlink(sp);
  unlink(lp);
  return 0;
}
