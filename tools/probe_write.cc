// Page-cache write bandwidth probe: one file of `gib` GiB written from a
// host buffer by (a) one write() stream, (b) T threads pwrite()ing disjoint
// ranges, (c) T threads memcpy()ing into a shared mmap of the file.
// usage: probe_write <path> <gib> <threads...>
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: probe_write path gib threads...\n"); return 1; }
  const char* path = argv[1];
  const size_t N = (size_t)(atof(argv[2]) * (1ull << 30));
  char* srcp = nullptr;
  if (posix_memalign((void**)&srcp, 4096, N)) return 1;
  struct { char* p; char* data() { return p; } } src{srcp};
  for (size_t i = 0; i < N; ++i) srcp[i] = "ACGT 0123456789\n"[i & 15];
  for (int a = 3; a < argc; ++a) {
    const int T = atoi(argv[a]);
    for (int mode = 0; mode < 6; ++mode) {
      if (mode == 0 && T != 1) continue;
      unlink(path);
      int fd = open(path, O_CREAT | O_RDWR | O_TRUNC | (mode >= 3 ? O_DIRECT : 0), 0644);
      if (fd < 0) { perror("open"); return 1; }
      // modes 4 / 5: the file sized first (fallocate / sparse ftruncate), so the direct
      // writes do not extend it (file systems may then take the inode lock shared)
      if (mode == 4 && fallocate(fd, 0, 0, (off_t)N)) { perror("fallocate"); return 1; }
      if (mode == 5 && ftruncate(fd, (off_t)N)) { perror("ftruncate"); return 1; }
      const double t0 = now();
      if (mode == 0) {
        size_t o = 0;
        while (o < N) { ssize_t w = write(fd, src.data() + o, std::min<size_t>(N - o, 64 << 20)); if (w <= 0) { perror("write"); return 1; } o += (size_t)w; }
      } else if (mode == 1) {
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
          th.emplace_back([&, t] {
            size_t a0 = N * t / T, a1 = N * (t + 1) / T;
            while (a0 < a1) { ssize_t w = pwrite(fd, src.data() + a0, std::min<size_t>(a1 - a0, 64 << 20), (off_t)a0); if (w <= 0) { perror("pwrite"); exit(1); } a0 += (size_t)w; }
          });
        for (auto& x : th) x.join();
      } else if (mode >= 3) {  // O_DIRECT pwrite of aligned 64 MiB pieces from T threads
        std::vector<std::thread> th;
        const size_t piece = 64 << 20;
        std::atomic<size_t> next(0);
        for (int t = 0; t < T; ++t)
          th.emplace_back([&] {
            for (;;) {
              const size_t o = next.fetch_add(piece);
              if (o >= N) break;
              const size_t len = std::min(piece, N - o) & ~(size_t)4095;
              if (!len) break;
              if (pwrite(fd, src.data() + o, len, (off_t)o) != (ssize_t)len) { perror("pwrite O_DIRECT"); exit(1); }
            }
          });
        for (auto& x : th) x.join();
      } else {
        if (ftruncate(fd, (off_t)N)) { perror("ftruncate"); return 1; }
        char* m = (char*)mmap(nullptr, N, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (m == MAP_FAILED) { perror("mmap"); return 1; }
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
          th.emplace_back([&, t] { size_t a0 = N * t / T, a1 = N * (t + 1) / T; memcpy(m + a0, src.data() + a0, a1 - a0); });
        for (auto& x : th) x.join();
        munmap(m, N);
      }
      close(fd);
      const double dt = now() - t0;
      static const char* names[] = {"write", "pwrite", "mmap", "odirect", "odirect_fallocated", "odirect_sized"};
      printf("%s threads=%d %.2f GB/s (%.3f s)\n", names[mode], T, N / dt / 1e9, dt);
      fflush(stdout);
    }
  }
  unlink(path);
  return 0;
}
