// --index-cache PATH for the CLIs (optional on-disk index
// cache).  The cache holds the built index (pbgpu_index_save); its tag names
// the index parameters and every super-read file's size and modification time,
// so a cache written for other inputs or parameters is rebuilt, never used.
#pragma once
#include <sys/stat.h>

#include <string>
#include <vector>

#include "../../include/pbgpu.h"

inline std::string index_cache_tag(const pbgpu_index_params& ip, const std::vector<const char*>& srs) {
  std::string t = "k=" + std::to_string(ip.k) + " psa_min=" + std::to_string(ip.psa_min) +
                  " fine_k=" + std::to_string(ip.fine_k) + " shard=" + std::to_string(ip.shard) + "/" +
                  std::to_string(ip.n_shards);
  for (const char* p : srs) {
    struct stat st {};
    t += std::string(" ") + p;
    if (stat(p, &st) == 0)
      t += ":" + std::to_string((long long)st.st_size) + ":" + std::to_string((long long)st.st_mtim.tv_sec) + "." +
           std::to_string((long long)st.st_mtim.tv_nsec);
  }
  return t;
}

// The index for `ip` from the cache when it matches, else built from `srs` and
// saved there (a failed save is reported and the run goes on).  Returns the
// status of the build (or of the load).
inline pbgpu_status index_from_cache(const char* cache, const std::vector<const char*>& srs,
                                     const pbgpu_index_params& ip, pbgpu_index** out, bool verbose) {
  const std::string tag = index_cache_tag(ip, srs);
  if (cache) {
    struct stat st {};
    if (stat(cache, &st) == 0) {
      if (pbgpu_index_load(cache, ip.device, tag.c_str(), out) == PBGPU_OK) {
        if (verbose) fprintf(stderr, "index: loaded from cache %s\n", cache);
        return PBGPU_OK;
      }
      fprintf(stderr, "index cache %s not used (%s); rebuilding\n", cache, pbgpu_last_error());
    }
  }
  const pbgpu_status s = pbgpu_index_build_fasta(srs.data(), srs.size(), &ip, out);
  if (s != PBGPU_OK || !cache) return s;
  if (pbgpu_index_save(*out, cache, tag.c_str()) != PBGPU_OK)
    fprintf(stderr, "index cache %s not written: %s\n", cache, pbgpu_last_error());
  else if (verbose)
    fprintf(stderr, "index: saved to cache %s\n", cache);
  return PBGPU_OK;
}
