#include "storage.h"

#include "trace.h"
#include "xet_hash.h"
#include "cdc.h"
#include <pthread.h>
#include <thread>

#include <dirent.h>
#include <signal.h>
#include <ctime>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cerrno>
#include <cstring>
#include <random>
#include <set>

#include "xorb.h"

namespace zest::storage {

void ensure_dir(const std::string& path) {
  if (path.empty()) return;
  std::string cur;
  size_t i = 0;
  if (path[0] == '/') {
    cur = "/";
    i = 1;
  }
  while (i <= path.size()) {
    size_t j = path.find('/', i);
    if (j == std::string::npos) j = path.size();
    if (j > i) {
      cur += path.substr(i, j - i);
      if (::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST)
        throw Error("IoError", "mkdir " + cur + ": " + std::strerror(errno));
      cur += "/";
    }
    i = j + 1;
  }
}

bool exists(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0;
}

uint64_t file_size(const std::string& path) {
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) return 0;
  return uint64_t(st.st_size);
}

void write_file_atomic(const std::string& path, const uint8_t* data, size_t n, bool durable) {
  const size_t slash = path.rfind('/');
  if (slash != std::string::npos) ensure_dir(path.substr(0, slash));
  static std::atomic<uint64_t> counter{0};
  const std::string tmp = path + ".tmp." + std::to_string(::getpid()) + "." + std::to_string(counter.fetch_add(1));
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) throw Error("IoError", "open " + tmp + ": " + std::strerror(errno));
  size_t off = 0;
  while (off < n) {
    ssize_t w = ::write(fd, data + off, std::min<size_t>(n - off, size_t(1) << 30));
    if (w < 0) {
      if (errno == EINTR) continue;
      ::close(fd);
      ::unlink(tmp.c_str());
      throw Error("IoError", "write " + tmp + ": " + std::strerror(errno));
    }
    off += size_t(w);
  }
  if (durable) ::fdatasync(fd);
  ::close(fd);
  if (::rename(tmp.c_str(), path.c_str()) != 0) {
    ::unlink(tmp.c_str());
    throw Error("IoError", "rename " + path + ": " + std::strerror(errno));
  }
}

std::optional<Bytes> read_file(const std::string& path) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return std::nullopt;
  struct stat st;
  if (::fstat(fd, &st) != 0) {
    ::close(fd);
    return std::nullopt;
  }
  Bytes out(size_t(st.st_size));
  size_t off = 0;
  while (off < out.size()) {
    ssize_t r = ::read(fd, out.data() + off, out.size() - off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) {
      ::close(fd);
      return std::nullopt;
    }
    off += size_t(r);
  }
  ::close(fd);
  return out;
}

bool read_range(const std::string& path, uint64_t off, uint64_t n, uint8_t* out) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  uint64_t got = 0;
  while (got < n) {
    ssize_t r = ::pread(fd, out + got, size_t(n - got), off_t(off + got));
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) break;
    got += uint64_t(r);
  }
  ::close(fd);
  return got == n;
}

void remove_file(const std::string& path) { ::unlink(path.c_str()); }

void start_writeback(int fd, uint64_t off, uint64_t len) {
  if (fd >= 0 && len) (void)::sync_file_range(fd, off64_t(off), off64_t(len), SYNC_FILE_RANGE_WRITE);
}

void write_ref(const Config& cfg, const std::string& repo_id, const std::string& ref, const std::string& commit) {
  write_file_atomic(cfg.repo_dir(repo_id) + "/refs/" + ref, commit);
}

std::optional<std::string> read_ref(const Config& cfg, const std::string& repo_id, const std::string& ref) {
  auto b = read_file(cfg.repo_dir(repo_id) + "/refs/" + ref);
  if (!b) return std::nullopt;
  std::string s(b->begin(), b->end());
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  return s;
}

std::vector<std::string> list_cached_xorbs(const Config& cfg) {
  std::set<std::string> out;
  DIR* d = ::opendir(cfg.xorb_cache_dir.c_str());
  if (!d) return {};
  while (dirent* e = ::readdir(d)) {
    std::string pfx = e->d_name;
    if (pfx.size() != 2) continue;
    DIR* sd = ::opendir((cfg.xorb_cache_dir + "/" + pfx).c_str());
    if (!sd) continue;
    while (dirent* f = ::readdir(sd)) {
      std::string n = f->d_name;
      if (n.size() < 64 || n.compare(0, 2, pfx) != 0) continue;
      // full `{hex}` or partial `{hex}.{digits}`; temp files and quarantined `.unverified` runs
      // are not cached xorbs
      if (n.size() == 64 || (n[64] == '.' && n.size() > 65 && std::all_of(n.begin() + 65, n.end(), ::isdigit)))
        out.insert(n.substr(0, 64));
    }
    ::closedir(sd);
  }
  ::closedir(d);
  return {out.begin(), out.end()};
}

void XorbRegistry::add(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  keys_.insert(key);
}
void XorbRegistry::remove(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  keys_.erase(key);
}
bool XorbRegistry::has(const std::string& key) const {
  std::lock_guard<std::mutex> g(mu_);
  return keys_.count(key) > 0;
}
size_t XorbRegistry::count() const {
  std::lock_guard<std::mutex> g(mu_);
  return keys_.size();
}
void XorbRegistry::scan(const Config& cfg) {
  auto l = list_cached_xorbs(cfg);
  std::lock_guard<std::mutex> g(mu_);
  for (auto& k : l) keys_.insert(k);
}
std::vector<std::string> XorbRegistry::keys() const {
  std::lock_guard<std::mutex> g(mu_);
  return {keys_.begin(), keys_.end()};
}

bool XorbCache::has(const std::string& hex) const { return exists(cfg_.xorb_cache_path(hex)); }

std::optional<Bytes> XorbCache::get(const std::string& hex) const { return read_file(cfg_.xorb_cache_path(hex)); }

std::optional<CacheHit> slice_run(const Bytes& data, uint32_t offset, uint32_t start, uint32_t end) {
  if (start < offset) return std::nullopt;
  std::vector<xet::ChunkEntry> idx;
  try {
    idx = xet::index_chunks(data.data(), data.size());
  } catch (const Error&) {
    return std::nullopt;
  }
  const uint64_t a = start - offset;
  const uint64_t b = end == 0 ? idx.size() : uint64_t(end) - offset;
  if (a >= b || b > idx.size()) return std::nullopt;
  const uint64_t lo = idx[a].header_off;
  const uint64_t hi = idx[b - 1].header_off + xet::kChunkHeaderLen + idx[b - 1].clen;
  CacheHit h;
  h.chunk_offset = start;
  if (lo == 0 && hi == data.size()) h.data = data;
  else h.data.assign(data.begin() + long(lo), data.begin() + long(hi));
  return h;
}

std::vector<uint32_t> XorbCache::run_offsets(const std::string& hex) const {
  std::vector<uint32_t> out;
  if (hex.size() != 64) return out;
  const std::string dir = cfg_.xorb_cache_dir + "/" + hex.substr(0, 2);
  DIR* d = ::opendir(dir.c_str());
  if (!d) return out;
  while (dirent* e = ::readdir(d)) {
    std::string n = e->d_name;
    if (n.compare(0, 64, hex) != 0) continue;
    if (n.size() == 64) {
      out.push_back(0);
    } else if (n[64] == '.' && n.size() > 65 && std::all_of(n.begin() + 65, n.end(), ::isdigit)) {
      out.push_back(uint32_t(std::stoul(n.substr(65))));
    }
  }
  ::closedir(d);
  std::sort(out.begin(), out.end());
  out.erase(std::unique(out.begin(), out.end()), out.end());
  return out;
}

namespace {
struct Mapping {
  void* p = MAP_FAILED;
  size_t n = 0;
  ~Mapping() {
    if (p != MAP_FAILED) ::munmap(p, n);
  }
};

// Map a cache file read-only; nullptr when missing / empty.
std::shared_ptr<Mapping> map_file(const std::string& path) {
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) return nullptr;
  struct stat st;
  if (::fstat(fd, &st) != 0 || st.st_size <= 0) {
    ::close(fd);
    return nullptr;
  }
  auto m = std::make_shared<Mapping>();
  m->n = size_t(st.st_size);
  m->p = ::mmap(nullptr, m->n, PROT_READ, MAP_SHARED, fd, 0);
  ::close(fd);
  if (m->p == MAP_FAILED) return nullptr;
  ::madvise(m->p, m->n, MADV_SEQUENTIAL);
  return m;
}
}  // namespace

// Identity of this process's pid namespace on this boot: a pid is only meaningful to kill() inside
// the namespace it came from.  Hash of the kernel boot id and the pid-namespace inode, 12 hex digits.
const std::string& pid_namespace_token() {
  static const std::string tok = [] {
    uint64_t h = 1469598103934665603ull;  // FNV-1a
    auto mix = [&](const std::string& s) {
      for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    };
    if (auto b = read_file("/proc/sys/kernel/random/boot_id")) mix(std::string(b->begin(), b->end()));
    struct stat st;
    if (::stat("/proc/self/ns/pid", &st) == 0) mix(std::to_string(uint64_t(st.st_ino)) + ":" + std::to_string(st.st_dev));
    char buf[17];
    std::snprintf(buf, sizeof buf, "%012llx", static_cast<unsigned long long>(h & 0xFFFFFFFFFFFFull));
    return std::string(buf);
  }();
  return tok;
}

// A quarantine file `{run}.p{pid}-{seq}-n{ns}.unverified` is stale when it is older than `max_age_s`
// (a pull never holds a run that long), or when its writer ran in this pid namespace and is gone (no
// process with that pid).  A writer in another namespace -- another container sharing the cache --
// is invisible to kill(), so only the age limit applies to its files.
bool stale_pending(const std::string& path, int64_t max_age_s) {
  const std::string suffix = XorbCache::kPendingSuffix;
  if (path.size() < suffix.size() || path.compare(path.size() - suffix.size(), suffix.size(), suffix) != 0)
    return false;
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) return false;
  if (max_age_s >= 0 && ::time(nullptr) - st.st_mtim.tv_sec > max_age_s) return true;
  const size_t p = path.rfind(".p");
  if (p == std::string::npos) return true;  // pre-round-3 name without a pid: nobody owns it
  const size_t ns = path.rfind("-n");
  if (ns != std::string::npos && ns > p) {
    const std::string tok = path.substr(ns + 2, path.size() - suffix.size() - (ns + 2));
    if (tok != pid_namespace_token()) return false;  // another namespace: age limit only
  }
  const long pid = std::strtol(path.c_str() + p + 2, nullptr, 10);
  if (pid <= 0) return true;
  return ::kill(pid_t(pid), 0) != 0 && errno == ESRCH;
}

// Zero-copy: the hit views the page-cache mapping of the run file (cache files are only ever
// replaced by rename, never truncated in place, so a live mapping stays valid).  Only the chunk
// headers are touched to validate coverage.
std::optional<CacheHit> XorbCache::find(const std::string& hex, uint32_t start, uint32_t end) const {
  if (registry_lookup_ && registry_ && !registry_->has(hex)) return std::nullopt;
  auto offs = run_offsets(hex);
  // Closest preceding run first: most likely to be the one that was fetched for this range.
  for (auto it = offs.rbegin(); it != offs.rend(); ++it) {
    if (*it > start) continue;
    const std::string path = cfg_.xorb_cache_path(*it == 0 ? hex : hex + "." + std::to_string(*it));
    auto m = map_file(path);
    if (!m) continue;
    const uint8_t* base = static_cast<const uint8_t*>(m->p);
    std::vector<xet::ChunkEntry> idx;
    try {
      idx = xet::index_chunks(base, m->n);
    } catch (const Error&) {
      continue;
    }
    const uint64_t a = start - *it;
    const uint64_t b = end == 0 ? idx.size() : uint64_t(end) - *it;
    if (a >= b || b > idx.size()) continue;
    const uint64_t lo = idx[a].header_off;
    const uint64_t hi = idx[b - 1].header_off + xet::kChunkHeaderLen + idx[b - 1].clen;
    CacheHit h;
    h.chunk_offset = start;
    h.run_offset = *it;
    h.ext = base + lo;
    h.ext_len = hi - lo;
    h.keep = m;
    (void)::utimensat(AT_FDCWD, path.c_str(), nullptr, 0);  // recently used: trim() keeps it longer
    return h;
  }
  return std::nullopt;
}

bool XorbCache::covers(const std::string& hex, uint32_t start, uint32_t end) const {
  if (end <= start) return false;
  if (registry_ && !registry_->has(hex) && run_offsets(hex).empty()) return false;
  for (uint32_t off : run_offsets(hex)) {
    if (off > start) continue;
    const std::string path = cfg_.xorb_cache_path(off == 0 ? hex : hex + "." + std::to_string(off));
    const int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) continue;
    struct stat st;
    const uint64_t size = ::fstat(fd, &st) == 0 ? uint64_t(st.st_size) : 0;
    (void)::posix_fadvise(fd, 0, 0, POSIX_FADV_RANDOM);
    uint64_t p = 0;
    uint32_t k = 0;
    const uint32_t need = end - off;
    bool ok = true;
    while (k < need) {
      uint8_t h[xet::kChunkHeaderLen];
      if (p + xet::kChunkHeaderLen > size || ::pread(fd, h, sizeof h, off_t(p)) != ssize_t(sizeof h)) {
        ok = false;
        break;
      }
      const uint64_t clen = uint64_t(h[1]) | uint64_t(h[2]) << 8 | uint64_t(h[3]) << 16;
      if (h[0] != 0 || h[4] > 2 || p + xet::kChunkHeaderLen + clen > size) {
        ok = false;
        break;
      }
      p += xet::kChunkHeaderLen + clen;
      ++k;
    }
    ::close(fd);
    if (ok) return true;
  }
  return false;
}

std::optional<CacheHit> XorbCache::get_with_range(const std::string& hex, uint32_t range_start) const {
  if (auto full = read_file(cfg_.xorb_cache_path(hex))) return CacheHit{std::move(*full), 0};
  if (auto part = read_file(cfg_.xorb_cache_path(hex + "." + std::to_string(range_start))))
    return CacheHit{std::move(*part), range_start};
  return std::nullopt;
}

std::string XorbCache::run_path(const std::string& hex, uint32_t chunk_offset) const {
  return cfg_.xorb_cache_path(chunk_offset == 0 ? hex : hex + "." + std::to_string(chunk_offset));
}

void XorbCache::put_run(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n, bool replace) {
  const std::string path = run_path(hex, chunk_offset);
  if (!replace && exists(path) && file_size(path) >= n) return;  // keep the longer run
  write_file_atomic(path, data, n, /*durable=*/false);
  if (registry_) registry_->add(hex);
}

std::string XorbCache::pending_path(const std::string& hex, uint32_t chunk_offset) const {
  // One quarantine file per fetch: `{run}.p{pid}-{seq}.unverified`.  Files are reconstructed
  // concurrently, so two fetches of the same run (from different peers) must not share a name:
  // promote() publishes exactly the bytes that belonged to the file that verified.
  static std::atomic<uint64_t> seq{0};
  return run_path(hex, chunk_offset) + ".p" + std::to_string(::getpid()) + "-" + std::to_string(seq.fetch_add(1)) +
         "-n" + pid_namespace_token() + kPendingSuffix;
}

void XorbCache::write_pending(const std::string& path, const uint8_t* data, size_t n) {
  write_file_atomic(path, data, n, /*durable=*/false);
}

std::string XorbCache::put_pending(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n) {
  const std::string path = pending_path(hex, chunk_offset);
  write_pending(path, data, n);
  return path;
}

bool XorbCache::promote(const std::string& hex, uint32_t chunk_offset, const std::string& pending) {
  if (pending.empty() || !exists(pending)) return false;
  const std::string path = run_path(hex, chunk_offset);
  const uint64_t n = file_size(pending);
  if (exists(path) && file_size(path) >= n) {  // a published run at least as long already exists
    remove_file(pending);
    return true;
  }
  if (::rename(pending.c_str(), path.c_str()) != 0) {
    remove_file(pending);
    return false;
  }
  if (registry_) registry_->add(hex);
  return true;
}

void XorbCache::discard_pending(const std::string& pending) {
  if (!pending.empty()) remove_file(pending);
}

void XorbCache::evict(const std::string& hex, uint32_t chunk_offset) { remove_file(run_path(hex, chunk_offset)); }

uint64_t XorbCache::trim(uint64_t max_bytes, int64_t pending_max_age_s) {
  struct Run {
    int64_t mtime_ns;
    uint64_t size;
    std::string hex, path;
  };
  std::vector<Run> runs;
  uint64_t total = 0;
  DIR* d = ::opendir(cfg_.xorb_cache_dir.c_str());
  if (!d) return 0;
  while (dirent* e = ::readdir(d)) {
    const std::string pfx = e->d_name;
    if (pfx.size() != 2) continue;
    const std::string sub = cfg_.xorb_cache_dir + "/" + pfx;
    DIR* sd = ::opendir(sub.c_str());
    if (!sd) continue;
    while (dirent* f = ::readdir(sd)) {
      const std::string n = f->d_name;
      if (n.size() < 64 || n.compare(0, 2, pfx) != 0) continue;
      const bool run = n.size() == 64 ||
                       (n[64] == '.' && n.size() > 65 && std::all_of(n.begin() + 65, n.end(), ::isdigit));
      if (!run) {  // quarantined (.unverified) runs left behind by a pull that died are removed
        if (stale_pending(sub + "/" + n, pending_max_age_s)) ::unlink((sub + "/" + n).c_str());
        continue;  // live quarantine and temporary files stay
      }
      struct stat st;
      const std::string path = sub + "/" + n;
      if (::stat(path.c_str(), &st) != 0) continue;
      runs.push_back({int64_t(st.st_mtim.tv_sec) * 1000000000ll + st.st_mtim.tv_nsec, uint64_t(st.st_size),
                      n.substr(0, 64), path});
      total += uint64_t(st.st_size);
    }
    ::closedir(sd);
  }
  ::closedir(d);
  if (total <= max_bytes) return 0;
  std::sort(runs.begin(), runs.end(), [](const Run& a, const Run& b) { return a.mtime_ns < b.mtime_ns; });
  const uint64_t target = max_bytes - max_bytes / 10;
  uint64_t removed = 0;
  std::set<std::string> touched;
  for (const Run& r : runs) {
    if (total - removed <= target) break;
    if (::unlink(r.path.c_str()) == 0) {
      removed += r.size;
      touched.insert(r.hex);
    }
  }
  if (registry_)
    for (const auto& hex : touched)
      if (run_offsets(hex).empty()) registry_->remove(hex);
  return removed;
}

size_t XorbCache::sweep_pending(int64_t max_age_s) {
  size_t removed = 0;
  DIR* d = ::opendir(cfg_.xorb_cache_dir.c_str());
  if (!d) return 0;
  while (dirent* e = ::readdir(d)) {
    const std::string pfx = e->d_name;
    if (pfx.size() != 2) continue;
    const std::string sub = cfg_.xorb_cache_dir + "/" + pfx;
    DIR* sd = ::opendir(sub.c_str());
    if (!sd) continue;
    while (dirent* f = ::readdir(sd)) {
      const std::string path = sub + "/" + f->d_name;
      if (stale_pending(path, max_age_s) && ::unlink(path.c_str()) == 0) ++removed;
    }
    ::closedir(sd);
  }
  ::closedir(d);
  return removed;
}

uint64_t XorbCache::bytes_on_disk() const {
  uint64_t t = 0;
  for (auto& k : list_cached_xorbs(cfg_)) t += file_size(cfg_.xorb_cache_path(k));
  return t;
}

std::string verified_marker_path(const Config& cfg, const std::string& repo_id, const std::string& commit,
                                 const std::string& path) {
  const std::string repo = cfg.repo_dir(repo_id);
  const size_t slash = repo.rfind('/');
  return cfg.cache_dir + "/verified/" + (slash == std::string::npos ? repo : repo.substr(slash + 1)) + "/" + commit +
         "/" + path;
}

namespace {
bool stat_file(const std::string& file, uint64_t& size, uint64_t& mtime_ns) {
  struct stat st;
  if (::stat(file.c_str(), &st) != 0) return false;
  size = uint64_t(st.st_size);
  mtime_ns = uint64_t(st.st_mtim.tv_sec) * 1000000000ull + uint64_t(st.st_mtim.tv_nsec);
  return true;
}
}  // namespace

void write_verified_marker(const Config& cfg, const std::string& repo_id, const std::string& commit,
                           const std::string& path, const std::string& xet_hex, const std::string& file) {
  uint64_t size = 0, mtime = 0;
  if (!stat_file(file, size, mtime)) return;
  write_file_atomic(verified_marker_path(cfg, repo_id, commit, path),
                    xet_hex + " " + std::to_string(size) + " " + std::to_string(mtime) + "\n", false);
}

bool check_verified_marker(const Config& cfg, const std::string& repo_id, const std::string& commit,
                           const std::string& path, const std::string& xet_hex, const std::string& file) {
  uint64_t size = 0, mtime = 0;
  if (!stat_file(file, size, mtime)) return false;
  auto b = read_file(verified_marker_path(cfg, repo_id, commit, path));
  if (!b) return false;
  const std::string want = xet_hex + " " + std::to_string(size) + " " + std::to_string(mtime) + "\n";
  return std::string(b->begin(), b->end()) == want;
}

std::string xet_hash_of_file(const std::string& file, int threads) {
  int fd = ::open(file.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) throw Error("IoError", "open " + file);
  struct stat st;
  if (::fstat(fd, &st) != 0) {
    ::close(fd);
    throw Error("IoError", "stat " + file);
  }
  const size_t n = size_t(st.st_size);
  const uint8_t* data = nullptr;
  void* m = MAP_FAILED;
  if (n) {
    m = ::mmap(nullptr, n, PROT_READ, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) {
      ::close(fd);
      throw Error("IoError", "mmap " + file);
    }
    ::madvise(m, n, MADV_SEQUENTIAL);
    data = static_cast<const uint8_t*>(m);
  }
  ::close(fd);
  std::vector<uint64_t> ends = n ? xet::chunk_ends(data, n) : std::vector<uint64_t>{};
  std::vector<xet::HashSize> leaves(ends.size());
  const int nt = threads > 0 ? threads : int(std::max(1u, std::min(16u, std::thread::hardware_concurrency())));
  std::atomic<size_t> next{0};
  auto work = [&]() {
    for (size_t i; (i = next.fetch_add(1)) < ends.size();) {
      const uint64_t a = i ? ends[i - 1] : 0;
      leaves[i] = {xet::chunk_hash(data + a, size_t(ends[i] - a)), ends[i] - a};
    }
  };
  std::vector<std::thread> ts;
  for (int t = 0; t < nt; ++t) ts.emplace_back(work);
  for (auto& t : ts) t.join();
  if (m != MAP_FAILED) ::munmap(m, n);
  return xet::to_hex(xet::file_hash(leaves));
}

}  // namespace zest::storage

namespace zest::storage {

CacheWriter::CacheWriter(XorbCache* cache, size_t max_bytes, int threads)
    : cache_(cache), max_bytes_(max_bytes), queues_(size_t(std::max(1, threads))) {
  for (int q = 0; q < int(queues_.size()); ++q) threads_.emplace_back([this, q] {
    pthread_setname_np(pthread_self(), "zest-cachewr");
    worker(q);
  });
  for (int k = 0; k < 2; ++k) copy_threads_.emplace_back([this] {
    pthread_setname_np(pthread_self(), "zest-cachecp");
    copier();
  });
}

CacheWriter::~CacheWriter() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : copy_threads_) t.join();  // copiers first: they queue writes
  cv_.notify_all();
  for (auto& t : threads_) t.join();  // workers drain their queues before leaving
}

void CacheWriter::copier() {
  while (true) {
    CopyJob j;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return stop_ || !copies_.empty(); });
      if (copies_.empty()) return;  // stop_ and drained
      j = std::move(copies_.front());
      copies_.pop_front();
      ++copy_busy_;
    }
    {
      trace::Span sp("cache", j.op.kind == Op::Pending ? "quarantine copy (writer)" : "run copy (writer)");
      j.op.data = take_buffer(j.n);
      j.op.data.assign(j.src, j.src + j.n);
    }
    // queued before the caller hears the bytes are copied: a promote/discard it queues after that
    // (same xorb, same writer) runs after this write
    push(std::move(j.op));
    j.on_copied();
    {
      std::lock_guard<std::mutex> g(mu_);
      --copy_busy_;
    }
    cv_.notify_all();  // writers waiting to stop re-check
    idle_cv_.notify_all();
  }
}

std::string CacheWriter::put_pending_ref(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n,
                                         std::function<void()> on_copied) {
  if (!reserve(n)) return "";
  CopyJob j{Op{Op::Pending, hex, cache_->pending_path(hex, chunk_offset), chunk_offset, false, {}}, data, n,
            std::move(on_copied)};
  std::string path = j.op.path;
  {
    std::lock_guard<std::mutex> g(mu_);
    copies_.push_back(std::move(j));
  }
  cv_.notify_all();
  return path;
}

bool CacheWriter::put_run_ref(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n,
                              bool replace, std::function<void()> on_copied) {
  if (!reserve(n)) return false;
  CopyJob j{Op{Op::Run, hex, "", chunk_offset, replace, {}}, data, n, std::move(on_copied)};
  {
    std::lock_guard<std::mutex> g(mu_);
    copies_.push_back(std::move(j));
  }
  cv_.notify_all();
  return true;
}

bool CacheWriter::reserve(size_t n) {
  std::lock_guard<std::mutex> g(mu_);
  if (in_flight_ + n > max_bytes_) {
    st_.dropped_bytes += n;
    return false;
  }
  in_flight_ += n;
  st_.queued_bytes += n;
  return true;
}

Bytes CacheWriter::take_buffer(size_t n) {
  std::lock_guard<std::mutex> g(mu_);
  // smallest pooled buffer that fits: its pages are already faulted in
  size_t best = pool_.size();
  for (size_t i = 0; i < pool_.size(); ++i)
    if (pool_[i].capacity() >= n && (best == pool_.size() || pool_[i].capacity() < pool_[best].capacity())) best = i;
  if (best == pool_.size()) return Bytes();
  Bytes b = std::move(pool_[best]);
  pool_bytes_ -= b.capacity();
  pool_[best] = std::move(pool_.back());
  pool_.pop_back();
  return b;
}

void CacheWriter::push(Op op) {
  // per-xorb order: every operation on one xorb goes to the same writer
  const size_t q = op.hex.empty() ? 0 : std::hash<std::string>{}(op.hex) % queues_.size();
  {
    std::lock_guard<std::mutex> g(mu_);
    queues_[q].push_back(std::move(op));
    st_.ops++;
  }
  cv_.notify_all();
}

bool CacheWriter::put_run(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n, bool replace) {
  if (!reserve(n)) return false;
  Op op{Op::Run, hex, "", chunk_offset, replace, take_buffer(n)};
  op.data.assign(data, data + n);
  push(std::move(op));
  return true;
}

std::string CacheWriter::put_pending(const std::string& hex, uint32_t chunk_offset, const uint8_t* data, size_t n) {
  if (!reserve(n)) return "";
  Op op{Op::Pending, hex, cache_->pending_path(hex, chunk_offset), chunk_offset, false, take_buffer(n)};
  op.data.assign(data, data + n);
  std::string path = op.path;
  push(std::move(op));
  return path;
}

void CacheWriter::promote(const std::string& hex, uint32_t chunk_offset, const std::string& pending) {
  push(Op{Op::Promote, hex, pending, chunk_offset, false, {}});
}
void CacheWriter::discard_pending(const std::string& pending) {
  // a quarantine path embeds its xorb's hex: same writer as the write it discards
  const size_t slash = pending.rfind('/');
  std::string hex = pending.substr(slash == std::string::npos ? 0 : slash + 1, 64);
  push(Op{Op::Discard, hex, pending, 0, false, {}});
}
void CacheWriter::evict(const std::string& hex, uint32_t chunk_offset) {
  push(Op{Op::Evict, hex, "", chunk_offset, false, {}});
}

void CacheWriter::flush() {
  std::unique_lock<std::mutex> g(mu_);
  idle_cv_.wait(g, [&] {
    if (busy_ || copy_busy_ || !copies_.empty()) return false;
    for (auto& q : queues_)
      if (!q.empty()) return false;
    return true;
  });
}

CacheWriter::Stats CacheWriter::stats() const {
  std::lock_guard<std::mutex> g(mu_);
  return st_;
}

void CacheWriter::worker(int q) {
  while (true) {
    Op op;
    {
      std::unique_lock<std::mutex> g(mu_);
      // (at stop: leave only once the copy threads can queue nothing more)
      cv_.wait(g, [&] { return !queues_[size_t(q)].empty() || (stop_ && copies_.empty() && !copy_busy_); });
      if (queues_[size_t(q)].empty()) return;  // stop_ and drained
      op = std::move(queues_[size_t(q)].front());
      queues_[size_t(q)].pop_front();
      ++busy_;
    }
    const size_t n = op.data.size();
    try {
      switch (op.kind) {
        case Op::Run: cache_->put_run(op.hex, op.offset, op.data.data(), n, op.replace); break;
        case Op::Pending: cache_->write_pending(op.path, op.data.data(), n); break;
        case Op::Promote: cache_->promote(op.hex, op.offset, op.path); break;
        case Op::Discard: cache_->discard_pending(op.path); break;
        case Op::Evict: cache_->evict(op.hex, op.offset); break;
      }
    } catch (const std::exception&) {
      // best effort, like the synchronous path (a failed cache write only costs a refetch)
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      if (n) {
        in_flight_ -= n;
        st_.written_bytes += n;
        op.data.clear();
        if (pool_bytes_ + op.data.capacity() <= max_bytes_) {  // pooled buffers stay within the bound
          pool_bytes_ += op.data.capacity();
          pool_.push_back(std::move(op.data));
        }
      }
      --busy_;
    }
    idle_cv_.notify_all();
  }
}

}  // namespace zest::storage
