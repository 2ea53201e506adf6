// Native webdataset tar-shard reader (host C++, pybind11 module ``jumbo_mae_tpu_amd._io``).
//
// Reference data path (/root/reference/src/dataset.py:107-116, 139-150): webdataset's
// ``tarfile_to_samples(handler=ignore_and_continue)`` parses every shard in Python inside each
// DataLoader worker.  Here the parsing and file I/O run on a pool of native threads (no GIL):
//
//  * ustar / GNU / pax tar parsing straight from an mmap of the shard: header checksum validated,
//    octal or base-256 sizes, GNU long names ('L'), pax ``path`` / ``size`` records ('x'), global
//    pax headers and non-regular members skipped;
//  * webdataset grouping: consecutive members with the same key (path up to the first '.' of the
//    basename) form one sample {ext: bytes}; members without an extension are ignored;
//  * ORDERED read-ahead: up to ``threads`` shards are parsed concurrently, but samples are handed
//    out in shard order, so the stream is identical to a sequential read (deterministic shuffles
//    downstream stay reproducible); each shard's pending samples are capped in bytes so read-ahead
//    memory is bounded;
//  * the error semantics of Python's tarfile stream reader + ``ignore_and_continue``: a shard that
//    is missing, empty, has a bad first header or member data past its end yields the samples
//    completed before the fault; the error is then counted and skipped (``ignore_errors``) or
//    raised as RuntimeError at that point of the stream.  A bad header after the first ends the
//    shard silently, as in tarfile.
//
// The consumer side (__next__) waits with the GIL released.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

namespace py = pybind11;

namespace {

struct Member {
  std::string name;
  size_t offset;  // of the data, in bytes from the start of the file
  size_t size;
};

// read-only mmap of a whole file (RAII)
class Mapped {
 public:
  explicit Mapped(const std::string& path) {
    fd_ = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd_ < 0) throw std::runtime_error("cannot open " + path + ": " + std::strerror(errno));
    struct stat st;
    if (::fstat(fd_, &st) != 0) {
      ::close(fd_);
      throw std::runtime_error("cannot stat " + path);
    }
    size_ = (size_t)st.st_size;
    if (size_ > 0) {
      void* p = ::mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
      if (p == MAP_FAILED) {
        ::close(fd_);
        throw std::runtime_error("cannot mmap " + path);
      }
      (void)::madvise(p, size_, MADV_SEQUENTIAL);
      data_ = static_cast<const uint8_t*>(p);
    }
  }
  ~Mapped() {
    if (data_) ::munmap(const_cast<uint8_t*>(data_), size_);
    if (fd_ >= 0) ::close(fd_);
  }
  Mapped(const Mapped&) = delete;
  Mapped& operator=(const Mapped&) = delete;
  const uint8_t* data() const { return data_; }
  size_t size() const { return size_; }

 private:
  int fd_ = -1;
  const uint8_t* data_ = nullptr;
  size_t size_ = 0;
};

// One webdataset sample: its members stay in the shard's mmap (kept alive by the shared pointer)
// until the consumer copies them into Python bytes -- one copy per member in total.
struct Field {
  std::string ext;
  size_t offset, size;
};

struct Sample {
  std::string key;
  std::shared_ptr<Mapped> map;
  std::vector<Field> fields;
  size_t bytes = 0;
};

std::string cstr_field(const uint8_t* p, size_t n) {
  size_t len = 0;
  while (len < n && p[len] != 0) ++len;
  return std::string(reinterpret_cast<const char*>(p), len);
}

// numeric header field: octal ASCII (space / NUL terminated) or GNU base-256 (high bit set)
uint64_t num_field(const uint8_t* p, size_t n) {
  if (p[0] & 0x80) {
    uint64_t v = p[0] & 0x7f;
    for (size_t i = 1; i < n; ++i) v = (v << 8) | p[i];
    return v;
  }
  uint64_t v = 0;
  size_t i = 0;
  while (i < n && (p[i] == ' ' || p[i] == 0)) ++i;
  for (; i < n && p[i] >= '0' && p[i] <= '7'; ++i) v = v * 8 + (p[i] - '0');
  return v;
}

bool zero_block(const uint8_t* p) {
  for (int i = 0; i < 512; ++i)
    if (p[i]) return false;
  return true;
}

bool checksum_ok(const uint8_t* h) {
  const uint64_t want = num_field(h + 148, 8);
  uint64_t sum = 0;
  for (int i = 0; i < 512; ++i) sum += (i >= 148 && i < 156) ? ' ' : h[i];
  return sum == want;
}

// pax extended header records: "<len> <key>=<value>\n"
void parse_pax(const uint8_t* p, size_t n, std::string& path, int64_t& size) {
  size_t i = 0;
  while (i < n) {
    size_t j = i, len = 0;
    while (j < n && p[j] >= '0' && p[j] <= '9') len = len * 10 + (p[j++] - '0');
    if (len == 0 || i + len > n || j >= n || p[j] != ' ') return;
    const std::string rec(reinterpret_cast<const char*>(p + j + 1), i + len - (j + 1));
    const size_t eq = rec.find('=');
    if (eq != std::string::npos) {
      std::string key = rec.substr(0, eq), val = rec.substr(eq + 1);
      if (!val.empty() && val.back() == '\n') val.pop_back();
      if (key == "path") path = val;
      else if (key == "size") size = std::stoll(val);
    }
    i += len;
  }
}

// Parse the regular-file members of a tar image with Python tarfile's stream semantics (what
// webdataset sees): an empty file or a bad / truncated FIRST header is an error; a bad or truncated
// header later on ends the archive silently; member data running past the end of the file is an
// error.  Members before a fault are reported through ``out`` first.
void parse_tar(const uint8_t* d, size_t n, std::vector<Member>& out) {
  if (n == 0) throw std::runtime_error("empty file");
  size_t off = 0;
  std::string long_name, pax_path;
  int64_t pax_size = -1;
  for (;;) {
    if (off + 512 > n) {
      if (off == 0) throw std::runtime_error("truncated header");
      return;
    }
    const uint8_t* h = d + off;
    if (zero_block(h)) return;  // end-of-archive marker
    if (!checksum_ok(h)) {
      if (off == 0) throw std::runtime_error("bad checksum");
      return;
    }
    const char type = (char)h[156];
    uint64_t size = num_field(h + 124, 12);
    if (type != 'x' && type != 'g' && pax_size >= 0) size = (uint64_t)pax_size;
    const size_t data = off + 512;
    if (data + size > n) throw std::runtime_error("truncated tar member at offset " + std::to_string(off));
    const size_t next = data + ((size + 511) / 512) * 512;
    if (type == 'L') {
      long_name = cstr_field(d + data, size);
    } else if (type == 'x') {
      parse_pax(d + data, size, pax_path, pax_size);
    } else if (type == 'g' || type == 'K') {
      // global pax header / GNU long link name: nothing we use
    } else {
      std::string name;
      if (!pax_path.empty()) {
        name = pax_path;
      } else if (!long_name.empty()) {
        name = long_name;
      } else {
        name = cstr_field(h, 100);
        const bool ustar = std::memcmp(h + 257, "ustar\0", 6) == 0;  // POSIX: prefix field valid
        if (ustar) {
          const std::string prefix = cstr_field(h + 345, 155);
          if (!prefix.empty()) name = prefix + "/" + name;
        }
      }
      if (type == '0' || type == '\0' || type == '7') out.push_back({name, data, (size_t)size});
      long_name.clear();
      pax_path.clear();
      pax_size = -1;
    }
    off = next;
  }
}

// webdataset key / extension split (data/shards.py _split_key): extension = after the first '.'
// of the basename; false if there is none
bool split_key(const std::string& name, std::string& key, std::string& ext) {
  const size_t slash = name.rfind('/');
  const size_t bstart = slash == std::string::npos ? 0 : slash + 1;
  const size_t dot = name.find('.', bstart);
  if (dot == std::string::npos) return false;
  key = name.substr(0, dot);
  ext = name.substr(dot + 1);
  std::transform(ext.begin(), ext.end(), ext.begin(), [](unsigned char c) { return (char)std::tolower(c); });
  return true;
}

class ShardReader {
 public:
  ShardReader(std::vector<std::string> paths, int threads, size_t slot_bytes, bool ignore_errors)
      : paths_(std::move(paths)),
        nthreads_(std::max(1, threads)),
        slot_bytes_(std::max<size_t>(slot_bytes, 1)),
        ignore_(ignore_errors) {
    for (int i = 0; i < nthreads_; ++i) pool_.emplace_back([this] { worker(); });
  }

  ~ShardReader() { close(); }

  void close() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_prod_.notify_all();
    cv_cons_.notify_all();
    for (auto& t : pool_)
      if (t.joinable()) t.join();
    pool_.clear();
  }

  // next sample in shard order; false at the end of the stream.  Throws (ignore_errors false) when
  // the stream reaches a shard error.
  bool next(Sample& s, std::string& url) {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      if (cur_ >= (int)paths_.size()) return false;
      Slot& sl = slots_[cur_];
      if (!sl.q.empty()) {
        s = std::move(sl.q.front());
        sl.q.pop_front();
        const bool was_full = sl.bytes >= slot_bytes_;
        sl.bytes -= s.bytes;
        url = paths_[cur_];
        lk.unlock();
        if (was_full) cv_prod_.notify_all();  // its producer may wait on the byte cap
        return true;
      }
      if (sl.done) {
        const std::string err = sl.err;
        const std::string bad = paths_[cur_];
        slots_.erase(cur_);
        ++cur_;
        lk.unlock();
        cv_prod_.notify_all();
        if (!err.empty()) {
          errors_.fetch_add(1);
          {
            std::lock_guard<std::mutex> g(err_mu_);
            last_error_ = bad + ": " + err;
          }
          if (!ignore_) throw std::runtime_error(bad + ": " + err);
        }
        lk.lock();
        continue;
      }
      cv_cons_.wait(lk);
    }
  }

  int errors() const { return errors_.load(); }
  std::string last_error() {
    std::lock_guard<std::mutex> g(err_mu_);
    return last_error_;
  }
  int num_shards() const { return (int)paths_.size(); }

 private:
  struct Slot {
    std::deque<Sample> q;
    size_t bytes = 0;
    bool done = false;
    std::string err;
  };

  void worker() {
    for (;;) {
      int j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        // claim the next shard within the read-ahead window of the consumer
        cv_prod_.wait(lk, [&] { return stop_ || claim_ >= (int)paths_.size() || claim_ < cur_ + nthreads_ + 1; });
        if (stop_ || claim_ >= (int)paths_.size()) return;
        j = claim_++;
        slots_[j];
      }
      std::string err;
      try {
        read_shard(j);
      } catch (const std::exception& e) {
        err = e.what();
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        auto it = slots_.find(j);
        if (it != slots_.end()) {
          it->second.done = true;
          it->second.err = err;
        }
      }
      cv_cons_.notify_all();
      cv_prod_.notify_all();
    }
  }

  // blocks while this shard's pending bytes exceed the cap (unless it is the consumer's shard,
  // which must always make progress); false when the reader is closing
  bool push(int j, Sample&& s) {
    std::unique_lock<std::mutex> lk(mu_);
    cv_prod_.wait(lk, [&] { return stop_ || j == cur_ || slots_[j].bytes < slot_bytes_; });
    if (stop_) return false;
    Slot& sl = slots_[j];
    sl.bytes += s.bytes;
    sl.q.push_back(std::move(s));
    const bool consumer_waits_here = j == cur_ && sl.q.size() == 1;
    lk.unlock();
    if (consumer_waits_here) cv_cons_.notify_one();
    return true;
  }

  void read_shard(int j) {
    auto m = std::make_shared<Mapped>(paths_[j]);
    std::vector<Member> members;
    std::string parse_err;
    try {
      parse_tar(m->data(), m->size(), members);
    } catch (const std::exception& e) {
      parse_err = e.what();  // members before the fault are still delivered
    }
    Sample cur;
    bool have = false;
    for (const Member& mb : members) {
      std::string key, ext;
      if (!split_key(mb.name, key, ext)) continue;
      if (have && cur.key != key) {
        if (!push(j, std::move(cur))) return;
        cur = Sample();
        have = false;
      }
      if (!have) {
        cur.key = key;
        cur.map = m;
        have = true;
      }
      cur.fields.push_back({ext, mb.offset, mb.size});
      cur.bytes += mb.size;
    }
    // a fault drops the sample being assembled, like the Python reader
    if (!parse_err.empty()) throw std::runtime_error(parse_err);
    if (have && !push(j, std::move(cur))) return;
  }

  std::vector<std::string> paths_;
  const int nthreads_;
  const size_t slot_bytes_;
  const bool ignore_;
  std::mutex mu_;
  std::condition_variable cv_prod_, cv_cons_;
  std::map<int, Slot> slots_;
  int claim_ = 0, cur_ = 0;
  bool stop_ = false;
  std::vector<std::thread> pool_;
  std::atomic<int> errors_{0};
  std::mutex err_mu_;
  std::string last_error_;
};

py::dict to_dict(Sample& s, const std::string& url) {
  py::dict d;
  d["__key__"] = s.key;
  d["__url__"] = url;
  const char* base = reinterpret_cast<const char*>(s.map->data());
  for (const Field& f : s.fields) d[py::str(f.ext)] = py::bytes(base + f.offset, f.size);
  return d;
}

py::list list_members(const std::string& path) {
  Mapped m(path);
  std::vector<Member> members;
  parse_tar(m.data(), m.size(), members);
  py::list out;
  for (const Member& mb : members) out.append(py::make_tuple(mb.name, mb.offset, mb.size));
  return out;
}

}  // namespace

PYBIND11_MODULE(_io, m) {
  m.doc() = "native webdataset tar-shard reader (ordered multi-threaded read-ahead)";
  m.def("list_members", &list_members, "regular-file members of a tar shard: [(name, data_offset, size)]");
  py::class_<ShardReader>(m, "ShardReader")
      .def(py::init<std::vector<std::string>, int, size_t, bool>(), py::arg("paths"), py::arg("threads") = 4,
           py::arg("slot_bytes") = (size_t)64 << 20, py::arg("ignore_errors") = false)
      .def("__iter__", [](ShardReader& r) -> ShardReader& { return r; })
      .def("__next__",
           [](ShardReader& r) {
             Sample s;
             std::string url;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = r.next(s, url);
             }
             if (!ok) throw py::stop_iteration();
             return to_dict(s, url);
           })
      .def("close", [](ShardReader& r) {
        py::gil_scoped_release nogil;
        r.close();
      })
      .def_property_readonly("errors", &ShardReader::errors)
      .def_property_readonly("last_error", &ShardReader::last_error)
      .def_property_readonly("num_shards", &ShardReader::num_shards);
}
