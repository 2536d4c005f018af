// TensorBoard event-file writer (MI355X-native replacement for TF1's C++ EventsWriter, which the
// reference drives through tf.summary.FileWriter / add_summary: R/distributed/distributed.py:138,151).
//
// * CRC32C (Castagnoli) with the SSE4.2 crc32 instruction (table fallback), TFRecord masking
//   ((crc >> 15 | crc << 17) + 0xa282ead8);
// * TFRecord framing: u64 len | u32 masked_crc(len) | data | u32 masked_crc(data);
// * Event protos hand-encoded (no protobuf dependency): field 1 wall_time (double), 2 step (int64),
//   3 file_version (string), 4 graph_def (bytes), 5 summary { value { 1 tag, 2 simple_value } };
// * a background thread drains a bounded queue and flushes, like TF's writer thread, so
//   add_summary() on the training loop costs one enqueue.
// C ABI for ctypes (tensorflow_examples_amd/summary).
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#if defined(__SSE4_2__)
#include <nmmintrin.h>
#endif

namespace {

uint32_t crc_table[8][256];
std::once_flag crc_once;

void init_table() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82f63b78u : (c >> 1);
    crc_table[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) crc_table[t][i] = (crc_table[t - 1][i] >> 8) ^ crc_table[0][crc_table[t - 1][i] & 0xff];
}

uint32_t crc32c_sw(uint32_t crc, const uint8_t* p, size_t n) {
  std::call_once(crc_once, init_table);
  crc = ~crc;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    crc = crc_table[0][(crc ^ *p++) & 0xff] ^ (crc >> 8);
    --n;
  }
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    v ^= crc;
    crc = crc_table[7][v & 0xff] ^ crc_table[6][(v >> 8) & 0xff] ^ crc_table[5][(v >> 16) & 0xff] ^
          crc_table[4][(v >> 24) & 0xff] ^ crc_table[3][(v >> 32) & 0xff] ^ crc_table[2][(v >> 40) & 0xff] ^
          crc_table[1][(v >> 48) & 0xff] ^ crc_table[0][(v >> 56) & 0xff];
    p += 8;
    n -= 8;
  }
  while (n--) crc = crc_table[0][(crc ^ *p++) & 0xff] ^ (crc >> 8);
  return ~crc;
}

#if defined(__SSE4_2__)
uint32_t crc32c_hw(uint32_t crc, const uint8_t* p, size_t n) {
  uint64_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}
#endif

uint32_t crc32c(const uint8_t* p, size_t n) {
#if defined(__SSE4_2__)
  return crc32c_hw(0, p, n);
#else
  return crc32c_sw(0, p, n);
#endif
}

uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

// ---------------------------------------------------------------- protobuf encoding helpers
void put_varint(std::string& s, uint64_t v) {
  while (v >= 0x80) {
    s.push_back((char)(v | 0x80));
    v >>= 7;
  }
  s.push_back((char)v);
}
void put_tag(std::string& s, int field, int wire) { put_varint(s, ((uint64_t)field << 3) | wire); }
void put_double(std::string& s, int field, double d) {
  put_tag(s, field, 1);
  char b[8];
  memcpy(b, &d, 8);
  s.append(b, 8);
}
void put_float(std::string& s, int field, float f) {
  put_tag(s, field, 5);
  char b[4];
  memcpy(b, &f, 4);
  s.append(b, 4);
}
void put_bytes(std::string& s, int field, const char* p, size_t n) {
  put_tag(s, field, 2);
  put_varint(s, n);
  s.append(p, n);
}
void put_int64(std::string& s, int field, int64_t v) {
  put_tag(s, field, 0);
  put_varint(s, (uint64_t)v);
}

std::string frame_record(const std::string& data) {
  std::string out;
  uint64_t len = data.size();
  char lb[8];
  memcpy(lb, &len, 8);
  out.append(lb, 8);
  uint32_t lc = mask_crc(crc32c(reinterpret_cast<const uint8_t*>(lb), 8));
  out.append(reinterpret_cast<const char*>(&lc), 4);
  out.append(data);
  uint32_t dc = mask_crc(crc32c(reinterpret_cast<const uint8_t*>(data.data()), data.size()));
  out.append(reinterpret_cast<const char*>(&dc), 4);
  return out;
}

struct Writer {
  FILE* f = nullptr;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::string> q;
  std::thread th;
  bool stop = false;
  bool busy = false;  // a popped record is being written (guarded by mu)
  double flush_secs = 2.0;
  std::atomic<uint64_t> written{0};

  void run() {
    auto last = std::chrono::steady_clock::now();
    std::unique_lock<std::mutex> lk(mu);
    while (true) {
      // system_clock deadline: libstdc++ maps it to pthread_cond_timedwait, which ThreadSanitizer
      // intercepts (a steady_clock wait_for becomes pthread_cond_clockwait, which GCC 11's TSAN
      // does not model -- it then reports the waiting mutex as held: tests/test_runtime_sanitizers.py)
      cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(200),
                    [&] { return stop || !q.empty(); });
      while (!q.empty()) {
        std::string rec = std::move(q.front());
        q.pop_front();
        busy = true;
        lk.unlock();
        fwrite(rec.data(), 1, rec.size(), f);
        written.fetch_add(1);
        lk.lock();
        busy = false;
      }
      auto now = std::chrono::steady_clock::now();
      if (stop || std::chrono::duration<double>(now - last).count() >= flush_secs) {
        fflush(f);
        last = now;
      }
      if (stop) break;
    }
  }
  void enqueue(std::string rec) {
    {
      std::lock_guard<std::mutex> g(mu);
      q.push_back(std::move(rec));
    }
    cv.notify_one();
  }
};

}  // namespace

extern "C" {

uint32_t tfx_crc32c(const uint8_t* p, size_t n) { return crc32c(p, n); }
uint32_t tfx_crc32c_sw(const uint8_t* p, size_t n) { return crc32c_sw(0, p, n); }
uint32_t tfx_masked_crc32c(const uint8_t* p, size_t n) { return mask_crc(crc32c(p, n)); }

void* tfx_events_open(const char* path, double wall_time) {
  FILE* f = fopen(path, "wb");
  if (!f) return nullptr;
  Writer* w = new Writer();
  w->f = f;
  // first record: file_version "brain.Event:2"
  std::string ev;
  put_double(ev, 1, wall_time);
  const char* ver = "brain.Event:2";
  put_bytes(ev, 3, ver, strlen(ver));
  std::string rec = frame_record(ev);
  fwrite(rec.data(), 1, rec.size(), f);
  fflush(f);
  w->th = std::thread([w] { w->run(); });
  return w;
}

// Summary event with n scalar values
void tfx_events_add_scalars(void* h, int64_t step, double wall_time, int n, const char** tags, const float* vals) {
  Writer* w = static_cast<Writer*>(h);
  std::string summary;
  for (int i = 0; i < n; ++i) {
    std::string val;
    put_bytes(val, 1, tags[i], strlen(tags[i]));
    put_float(val, 2, vals[i]);
    put_bytes(summary, 1, val.data(), val.size());
  }
  std::string ev;
  put_double(ev, 1, wall_time);
  put_int64(ev, 2, step);
  put_bytes(ev, 5, summary.data(), summary.size());
  w->enqueue(frame_record(ev));
}

// Event carrying a serialized GraphDef (field 4) or any raw pre-encoded Event (raw=1)
void tfx_events_add_bytes(void* h, int64_t step, double wall_time, int field, const char* data, size_t n) {
  Writer* w = static_cast<Writer*>(h);
  std::string ev;
  put_double(ev, 1, wall_time);
  put_int64(ev, 2, step);
  put_bytes(ev, field, data, n);
  w->enqueue(frame_record(ev));
}

void tfx_events_add_record(void* h, const char* data, size_t n) {
  static_cast<Writer*>(h)->enqueue(frame_record(std::string(data, n)));
}

void tfx_events_flush(void* h) {
  Writer* w = static_cast<Writer*>(h);
  // wait for the queue to drain, then fflush
  for (int i = 0; i < 5000; ++i) {
    {
      std::lock_guard<std::mutex> g(w->mu);
      if (w->q.empty() && !w->busy) break;
    }
    w->cv.notify_one();
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  std::lock_guard<std::mutex> g(w->mu);
  fflush(w->f);
}

uint64_t tfx_events_written(void* h) { return static_cast<Writer*>(h)->written.load(); }

void tfx_events_close(void* h) {
  Writer* w = static_cast<Writer*>(h);
  {
    std::lock_guard<std::mutex> g(w->mu);
    w->stop = true;
  }
  w->cv.notify_one();
  w->th.join();
  fclose(w->f);
  delete w;
}

// Standalone TFRecord writer (checkpoint meta / generic records)
int tfx_tfrecord_append(const char* path, const char* data, size_t n) {
  FILE* f = fopen(path, "ab");
  if (!f) return -1;
  std::string rec = frame_record(std::string(data, n));
  size_t wr = fwrite(rec.data(), 1, rec.size(), f);
  fclose(f);
  return wr == rec.size() ? 0 : -1;
}

}  // extern "C"

extern "C" int tfx_rt_version() { return 2; }
