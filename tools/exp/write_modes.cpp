// Output-file write rates on this box: write() from one thread, pwrite() from T threads,
// and a shared mapping filled by T threads (ftruncate, MADV_POPULATE_WRITE, memcpy).
//   g++ -O2 -pthread write_modes.cpp -o write_modes && ./write_modes DIR GB THREADS
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const size_t bytes = (size_t)(atof(argc > 2 ? argv[2] : "4") * (1ull << 30));
  const int T = argc > 3 ? atoi(argv[3]) : 8;
  const size_t chunk = 64ull << 20;
  std::vector<char> src(chunk);
  for (size_t i = 0; i < chunk; ++i) src[i] = (char)('a' + i % 23);
  const std::string path = dir + "/write_modes.tmp";
  auto run = [&](const char* name, auto body) {
    unlink(path.c_str());
    int fd = open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0644);
    const double t0 = now();
    body(fd);
    close(fd);
    const double t = now() - t0;
    printf("%-28s %6.3f s  %6.2f GB/s\n", name, t, bytes / t / 1e9);
    fflush(stdout);
  };
  run("write 1 thread", [&](int fd) {
    for (size_t o = 0; o < bytes; o += chunk) if (write(fd, src.data(), std::min(chunk, bytes - o)) < 0) abort();
  });
  for (int t : {2, 4, T}) {
    char nm[64]; snprintf(nm, sizeof nm, "pwrite %d threads", t);
    run(nm, [&](int fd) {
      std::vector<std::thread> th;
      for (int k = 0; k < t; ++k)
        th.emplace_back([&, k] {
          for (size_t o = (size_t)k * chunk; o < bytes; o += (size_t)t * chunk)
            if (pwrite(fd, src.data(), std::min(chunk, bytes - o), (off_t)o) < 0) abort();
        });
      for (auto& x : th) x.join();
    });
  }
  for (int t : {1, 4, T}) {
    char nm[64]; snprintf(nm, sizeof nm, "mmap %d threads", t);
    run(nm, [&](int fd) {
      if (ftruncate(fd, (off_t)bytes)) abort();
      char* m = (char*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      if (m == MAP_FAILED) abort();
      std::vector<std::thread> th;
      for (int k = 0; k < t; ++k)
        th.emplace_back([&, k] {
          for (size_t o = (size_t)k * chunk; o < bytes; o += (size_t)t * chunk) {
            const size_t n = std::min(chunk, bytes - o);
            madvise(m + o, n, MADV_POPULATE_WRITE);
            memcpy(m + o, src.data(), n);
          }
        });
      for (auto& x : th) x.join();
      munmap(m, bytes);
    });
  }
  unlink(path.c_str());
  return 0;
}
