// Filesystem layer: atomic writes, HF cache layout (refs/snapshots), the content-addressed xorb
// disk cache and the xorb registry (piece map of what this node can seed).
//
// Reference: src/storage.zig:1-228 and XorbCache in src/swarm.zig:46-148.  Same on-disk names
// (xorbs/{hex[0..2]}/{hex} for full xorbs, {hex}.{range_start} for partial entries) but writes are
// really atomic (tmp + fsync + rename; the reference's writeFileAtomic is not, storage.zig:29-41),
// the registry is updated on every put (seed-while-downloading) and thread-safe.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "config.h"

namespace zest::storage {

void ensure_dir(const std::string& path);
bool exists(const std::string& path);
uint64_t file_size(const std::string& path);  // 0 if missing
// Write to a temp file and rename over `path`.  durable=false skips fdatasync (cache files: they
// are re-validated on read and content-verified by hash, so losing one on a crash only costs a
// refetch, while syncing every 64 MiB xorb serialises the pull on disk writeback).
void write_file_atomic(const std::string& path, const uint8_t* data, size_t n, bool durable = true);
inline void write_file_atomic(const std::string& path, const std::string& s, bool durable = true) {
  write_file_atomic(path, reinterpret_cast<const uint8_t*>(s.data()), s.size(), durable);
}
std::optional<Bytes> read_file(const std::string& path);
// Read [off, off+n) of a file into out (false if short/missing).
bool read_range(const std::string& path, uint64_t off, uint64_t n, uint8_t* out);
void remove_file(const std::string& path);
// Start the disk write-back of [off, off + len) of fd now (sync_file_range WRITE, no wait): the
// final fdatasync before a file's rename then only waits for what is still in flight, instead of
// flushing the whole file in the pull's tail.  Best effort (filesystems without it ignore it).
void start_writeback(int fd, uint64_t off, uint64_t len);

// HF cache: models--org--name/refs/{ref} = commit
void write_ref(const Config& cfg, const std::string& repo_id, const std::string& ref, const std::string& commit);
std::optional<std::string> read_ref(const Config& cfg, const std::string& repo_id, const std::string& ref);

// Distinct xorb hashes (hex) with any cached run: full `{hex}` or partial `{hex}.{chunk_offset}`.
std::vector<std::string> list_cached_xorbs(const Config& cfg);

struct CacheHit {
  Bytes data;
  uint32_t chunk_offset = 0;  // chunk index of data's first chunk inside the xorb
  uint32_t run_offset = 0;    // first chunk of the cached run the hit was sliced from (its file name)
  // Zero-copy alternative to `data` (e.g. a pinned staging buffer filled from HBM), valid while
  // `keep` is held.
  const uint8_t* ext = nullptr;
  size_t ext_len = 0;
  std::shared_ptr<void> keep;
  // A view still being filled (e.g. HBM -> pinned copies in flight): ready(n) blocks until bytes
  // [0, n) of `ext` are valid.  Empty: all of it is.  A server sends slice by slice behind it, so
  // the copy of one slice overlaps the send of the previous one.
  std::function<void(size_t)> ready;
  const uint8_t* bytes() const { return ext ? ext : data.data(); }
  size_t size() const { return ext ? ext_len : data.size(); }
  void wait_all() {
    if (ready) {
      ready(ext_len);
      ready = nullptr;
    }
  }
  void materialize() {  // copy an external view into `data`
    wait_all();
    if (ext) {
      data.assign(ext, ext + ext_len);
      ext = nullptr;
      ext_len = 0;
      keep.reset();
    }
  }
};

// Slice a run (first chunk = `offset`) to chunks [start, end); nullopt if it does not cover them.
std::optional<CacheHit> slice_run(const Bytes& data, uint32_t offset, uint32_t start, uint32_t end);

// Verified-file markers: `{cache_dir}/verified/{repo folder}/{commit}/{path}` holds
// "<xet hash> <size> <mtime ns>".  A snapshot file counts as cached only when its marker matches
// (the reference trusts existence alone, so a truncated file from a crash stays "cached" forever).
std::string verified_marker_path(const Config& cfg, const std::string& repo_id, const std::string& commit,
                                 const std::string& path);
void write_verified_marker(const Config& cfg, const std::string& repo_id, const std::string& commit,
                           const std::string& path, const std::string& xet_hex, const std::string& file);
bool check_verified_marker(const Config& cfg, const std::string& repo_id, const std::string& commit,
                           const std::string& path, const std::string& xet_hex, const std::string& file);
// Xet file hash of a file on disk (CDC + keyed BLAKE3 chunk hashes + Merkle), multi-threaded.
std::string xet_hash_of_file(const std::string& file, int threads = 0);

// A quarantine file whose writer died (pid gone) or older than max_age_s.
bool stale_pending(const std::string& path, int64_t max_age_s);

class XorbRegistry {
 public:
  void add(const std::string& key);
  void remove(const std::string& key);
  bool has(const std::string& key) const;
  size_t count() const;
  void scan(const Config& cfg);
  std::vector<std::string> keys() const;

 private:
  mutable std::mutex mu_;
  std::set<std::string> keys_;
};

class XorbCache {
 public:
  explicit XorbCache(const Config& cfg, XorbRegistry* registry = nullptr) : cfg_(cfg), registry_(registry) {}
  bool has(const std::string& hex) const;
  std::optional<Bytes> get(const std::string& hex) const;
  // A cached run covering chunks [start, end) (end == 0: through the end of the run), sliced to
  // exactly that range.  Every candidate is validated by walking its chunk headers, so a run
  // stored under the "full" name that is really a prefix (what the reference's
  // `range.start == 0 && one fetch entry` rule produces, xet_bridge.zig:189-217 — the source of
  // its P2P RangeOutOfBounds failures) is never served for chunks it does not hold.
  std::optional<CacheHit> find(const std::string& hex, uint32_t start, uint32_t end) const;
  // Pull pipelines whose registry was scanned at start: find() answers "not cached" from the
  // registry (what was cached at the scan + what this process published since) without listing the
  // xorb's cache directory, which a concurrent write-behind makes slow (4 ms per term in a 16-thread
  // device pull).  Runs another process adds during the pull are not seen -- they would only have
  // saved a fetch.  Servers keep the directory lookup.
  void set_registry_lookup(bool on) { registry_lookup_ = on; }
  // false: find() would answer "not cached" from the registry alone (no lookup worth tracing)
  bool maybe_cached(const std::string& hex) const { return !(registry_lookup_ && registry_ && !registry_->has(hex)); }
  // Does a cached run cover chunks [start, end)?  The planner's possession check (swarm_pull): only
  // the chunk headers up to `end` are read (pread, no readahead of the payload), and nothing is
  // mapped or touched.  A true answer is re-validated by find() when the term is fetched.
  bool covers(const std::string& hex, uint32_t start, uint32_t end) const;
  // Legacy lookup kept for callers that want the raw run at an exact offset.
  std::optional<CacheHit> get_with_range(const std::string& hex, uint32_t range_start) const;
  // Store a run of serialized chunks starting at chunk `chunk_offset`: offset 0 goes to `{hex}`,
  // others to `{hex}.{offset}`; an existing longer run under the same name is kept unless
  // `replace` (a CDN refetch repairing a cached copy that failed verification).
  void put_run(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n, bool replace = false);
  // Runs that nothing has verified yet (received from a peer) are quarantined under
  // `{run name}.unverified`, which no lookup, listing or seeding path sees.  After the file hash
  // checked out, promote() publishes the run (keeping an existing longer one); otherwise
  // discard_pending() drops it.  The reference caches peer runs unverified (swarm.zig:416-420) and
  // then serves them on; it caches only CDN bytes in the bridge (xet_bridge.zig:203-208).
  // put_pending returns the quarantine file's path (unique per call), which promote/discard take.
  std::string put_pending(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n);
  bool promote(const std::string& hex, uint32_t chunk_offset, const std::string& pending);
  void discard_pending(const std::string& pending);
  // Drop a published run (a cached copy whose bytes failed verification).
  void evict(const std::string& hex, uint32_t chunk_offset);
  static constexpr const char* kPendingSuffix = ".unverified";
  void put(const std::string& hex, const uint8_t* data, size_t n) { put_run(hex, 0, data, n); }
  void put_partial(const std::string& hex, uint32_t range_start, const uint8_t* data, size_t n) {
    put_run(hex, range_start, data, n);
  }
  std::vector<uint32_t> run_offsets(const std::string& hex) const;  // offsets of cached runs
  uint64_t bytes_on_disk() const;
  // Size bound (ZEST_CACHE_MAX_GB): when the published runs exceed `max_bytes`, delete the least
  // recently used ones (cache hits refresh a run's mtime) down to 90 % of it; xorbs with no run
  // left leave the registry, so they are no longer seeded.  Live quarantine and temporary files are
  // never touched; quarantine files whose writer process is gone, or older than
  // `pending_max_age_s` (< 0: no age limit), are deleted.  Returns the bytes of published runs
  // removed.  The reference's cache only grows.
  uint64_t trim(uint64_t max_bytes, int64_t pending_max_age_s = 24 * 3600);
  // Delete stale quarantine files only (see stale_pending); returns how many.  Runs after every
  // pull, so runs orphaned by a killed pull do not pile up outside the cache bound.
  size_t sweep_pending(int64_t max_age_s = 24 * 3600);

  // Quarantine file name for a new pending run (what put_pending writes to).
  std::string pending_path(const std::string& hex, uint32_t chunk_offset) const;
  void write_pending(const std::string& path, const uint8_t* data, size_t n);

 private:
  std::string run_path(const std::string& hex, uint32_t chunk_offset) const;
  const Config& cfg_;
  XorbRegistry* registry_;
  bool registry_lookup_ = false;
};

// Write-behind for the xorb cache.  A device pull moves tens of GB/s; writing every fetched run to
// disk on the fetch threads (8.3 ms per 64 MiB peer run in round 4's trace) put the disk in front of
// the H2D copy.  Here a fetch thread copies the run into a pooled buffer and returns; `threads`
// writers drain the queue in per-xorb FIFO order (a promote/discard/evict queued after a write of
// the same xorb runs after it).  The queue is bounded by `max_bytes`: when it is full a run is not
// cached at all (counted in `dropped_bytes`) -- the cache is best effort, the pull never waits on
// the disk.  The reference writes synchronously on the fetch task (swarm.zig:416-420,
// xet_bridge.zig:203-208).  The destructor drains the queue.
class CacheWriter {
 public:
  CacheWriter(XorbCache* cache, size_t max_bytes, int threads = 2);
  ~CacheWriter();
  CacheWriter(const CacheWriter&) = delete;
  CacheWriter& operator=(const CacheWriter&) = delete;
  // false: dropped (queue full)
  bool put_run(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n, bool replace);
  // The quarantine path the run will be written to, or "" when dropped.
  std::string put_pending(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n);
  // The same without copying on the caller's thread: `data` stays valid until on_copied() runs on
  // one of the writer's copy threads (which copy the run into a pooled buffer and queue its write;
  // the device pull keeps the pinned staging slot holding the run until then).  on_copied runs
  // exactly once when the call returns a path / true, never when it drops the run.
  std::string put_pending_ref(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n,
                              std::function<void()> on_copied);
  bool put_run_ref(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n, bool replace,
                   std::function<void()> on_copied);
  void promote(const std::string& hex, uint32_t chunk_offset, const std::string& pending);
  void discard_pending(const std::string& pending);
  void evict(const std::string& hex, uint32_t chunk_offset);
  void flush();  // wait until every queued operation ran
  struct Stats {
    uint64_t queued_bytes = 0, written_bytes = 0, dropped_bytes = 0, ops = 0;
  };
  Stats stats() const;

 private:
  struct Op {
    enum Kind { Run, Pending, Promote, Discard, Evict } kind;
    std::string hex, path;
    uint32_t offset = 0;
    bool replace = false;
    Bytes data;
  };
  struct CopyJob {
    Op op;  // data empty: copied from `src` by a copy thread
    const uint8_t* src = nullptr;
    size_t n = 0;
    std::function<void()> on_copied;
  };
  bool reserve(size_t n);
  Bytes take_buffer(size_t n);
  void push(Op op);
  void worker(int q);
  void copier();
  std::deque<CopyJob> copies_;
  size_t copy_busy_ = 0;
  std::vector<std::thread> copy_threads_;
  XorbCache* cache_;
  size_t max_bytes_;
  mutable std::mutex mu_;
  std::condition_variable cv_, idle_cv_;
  std::vector<std::deque<Op>> queues_;
  std::vector<Bytes> pool_;  // buffers of written runs, reused (no page faults on the fetch path)
  size_t pool_bytes_ = 0;
  size_t in_flight_ = 0;     // queued + being written (bytes)
  size_t busy_ = 0;          // operations popped and not finished
  bool stop_ = false;
  Stats st_;
  std::vector<std::thread> threads_;
};

}  // namespace zest::storage
