#include "storage.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstring>
#include <random>

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

void write_file_atomic(const std::string& path, const uint8_t* data, size_t n) {
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
  ::fdatasync(fd);
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
  std::vector<std::string> out;
  DIR* d = ::opendir(cfg.xorb_cache_dir.c_str());
  if (!d) return out;
  while (dirent* e = ::readdir(d)) {
    std::string pfx = e->d_name;
    if (pfx.size() != 2) continue;
    DIR* sd = ::opendir((cfg.xorb_cache_dir + "/" + pfx).c_str());
    if (!sd) continue;
    while (dirent* f = ::readdir(sd)) {
      std::string n = f->d_name;
      if (n.size() == 64 && n.compare(0, 2, pfx) == 0) out.push_back(n);
    }
    ::closedir(sd);
  }
  ::closedir(d);
  return out;
}

void XorbRegistry::add(const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  keys_.insert(key);
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

std::optional<CacheHit> XorbCache::get_with_range(const std::string& hex, uint32_t range_start) const {
  if (auto full = read_file(cfg_.xorb_cache_path(hex))) return CacheHit{std::move(*full), 0};
  if (auto part = read_file(cfg_.xorb_cache_path(hex + "." + std::to_string(range_start))))
    return CacheHit{std::move(*part), range_start};
  return std::nullopt;
}

void XorbCache::put(const std::string& hex, const uint8_t* data, size_t n) {
  write_file_atomic(cfg_.xorb_cache_path(hex), data, n);
  if (registry_) registry_->add(hex);
}

void XorbCache::put_partial(const std::string& hex, uint32_t range_start, const uint8_t* data, size_t n) {
  write_file_atomic(cfg_.xorb_cache_path(hex + "." + std::to_string(range_start)), data, n);
  if (registry_) registry_->add(hex + "." + std::to_string(range_start));
}

uint64_t XorbCache::bytes_on_disk() const {
  uint64_t t = 0;
  for (auto& k : list_cached_xorbs(cfg_)) t += file_size(cfg_.xorb_cache_path(k));
  return t;
}

}  // namespace zest::storage
