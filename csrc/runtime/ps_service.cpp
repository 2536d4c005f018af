// Parameter-server service: the MI355X-native replacement for the TF1 gRPC master/worker services
// that the reference's async-PS training runs on (tf.train.Server, R/distributed/distributed.py:41-43;
// server.join() :58; the per-step RecvTensor/RunGraph traffic of sess.run :148-150).
//
// One TCP service per ps task hosts NAMED f32 variables (round-robin sharded by the workers in
// creation order, like replica_device_setter).  A worker step is ONE round trip per ps task for
// the pull (all of that task's variables in one message) and ONE for push+apply+step-increment,
// instead of one RPC per tensor.  Updates are Hogwild/lock-free like TF's default
// ApplyGradientDescent(use_locking=False): elements are read/written with relaxed 32-bit atomics,
// so concurrent workers never tear a word (no data race in the C++ memory model) but may lose
// each other's updates, exactly the reference's async semantics.  Optional per-variable locking.
//
// Wire format (little endian):
//   request  : u32 magic 'TFPS' | u32 op | u32 n | f32 lr | u32 flags | n x item
//              item = u16 name_len | name | u64 nbytes | payload (ops CREATE, PUSH, ASSIGN only)
//   response : u32 status | u32 n | f64 scalar | n x (u64 nbytes | payload)   (PULL only)
// C ABI for ctypes (tensorflow_examples_amd/cluster/ps.py).
#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <stdint.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <memory>
#include <mutex>
#include <new>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

constexpr uint32_t MAGIC = 0x53504654;  // 'TFPS'
// Largest payload one item may carry.  The wire's u64 nbytes is untrusted: a larger value closes
// the connection instead of resizing a buffer to it (an uncaught bad_alloc would end the ps).
constexpr uint64_t MAX_ITEM_BYTES = 1ull << 31;
constexpr uint32_t STATUS_SIZE_MISMATCH = 0x80000000u;  // CREATE / ASSIGN: existing var, other size
enum Op : uint32_t {
  OP_PING = 0,
  OP_CREATE = 1,      // create + initialize if uninitialized (flags&1: force re-init = chief restart)
  OP_UNINIT = 2,      // count of uninitialized names (report_uninitialized_variables)
  OP_PULL = 3,
  OP_PUSH = 4,        // p -= lr * g for each item; flags&2: then increment "global_step" by 1
  OP_INC = 5,         // increment the single named scalar by lr (as delta); returns new value
  OP_ASSIGN = 6,
  OP_SHUTDOWN = 7,
  OP_STATS = 8,
};

struct Var {
  std::vector<uint32_t> bits;  // f32 payload accessed with relaxed atomics
  std::atomic<bool> init{false};
  std::mutex mu;               // used only when the service runs with use_locking
};

inline float ld(uint32_t* p) {
  uint32_t u = __atomic_load_n(p, __ATOMIC_RELAXED);
  float f;
  memcpy(&f, &u, 4);
  return f;
}
inline void st(uint32_t* p, float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  __atomic_store_n(p, u, __ATOMIC_RELAXED);
}

bool read_full(int fd, void* buf, size_t n) {
  char* p = static_cast<char*>(buf);
  while (n) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= (size_t)r;
  }
  return true;
}
bool write_full(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    ssize_t r = ::send(fd, p, n, MSG_NOSIGNAL);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= (size_t)r;
  }
  return true;
}

struct Server {
  int listen_fd = -1;
  int port = 0;
  bool use_locking = false;
  std::atomic<bool> stop{false};
  std::thread acceptor;
  std::mutex conn_mu;
  std::vector<std::thread> conns;
  std::vector<int> conn_fds;
  std::shared_mutex map_mu;
  std::unordered_map<std::string, std::unique_ptr<Var>> vars;
  std::atomic<uint64_t> n_pull{0}, n_push{0}, bytes_in{0}, bytes_out{0};

  Var* find(const std::string& name) {
    std::shared_lock<std::shared_mutex> g(map_mu);
    auto it = vars.find(name);
    return it == vars.end() ? nullptr : it->second.get();
  }
  Var* find_or_create(const std::string& name, size_t nfloat) {
    {
      std::shared_lock<std::shared_mutex> g(map_mu);
      auto it = vars.find(name);
      if (it != vars.end()) return it->second.get();
    }
    std::unique_lock<std::shared_mutex> g(map_mu);
    auto& slot = vars[name];
    if (!slot) {
      slot.reset(new Var());
      slot->bits.assign(nfloat, 0u);
    }
    return slot.get();
  }

  void handle(int fd) {
    std::vector<char> payload;
    while (!stop.load()) {
      uint32_t hdr[5];
      if (!read_full(fd, hdr, sizeof(hdr))) break;
      if (hdr[0] != MAGIC) break;
      const uint32_t op = hdr[1], n = hdr[2], flags = hdr[4];
      float lr;
      memcpy(&lr, &hdr[3], 4);
      uint32_t status = 0;
      double scalar = 0.0;
      std::vector<std::pair<const uint32_t*, uint64_t>> outs;  // PULL response pieces
      std::vector<std::vector<uint32_t>> snap;                   // PULL snapshots
      bool ok = true;
      for (uint32_t i = 0; i < n && ok; ++i) {
        uint16_t nl;
        if (!read_full(fd, &nl, 2)) { ok = false; break; }
        std::string name(nl, '\0');
        if (nl && !read_full(fd, &name[0], nl)) { ok = false; break; }
        uint64_t nbytes;
        if (!read_full(fd, &nbytes, 8)) { ok = false; break; }
        const bool carries = (op == OP_CREATE || op == OP_PUSH || op == OP_ASSIGN);
        if (carries) {
          if (nbytes > MAX_ITEM_BYTES) { ok = false; break; }
          try {
            payload.resize(nbytes);
          } catch (const std::bad_alloc&) {
            ok = false;
            break;
          }
          if (nbytes && !read_full(fd, payload.data(), nbytes)) { ok = false; break; }
          bytes_in += nbytes;
        }
        const size_t nf = nbytes / 4;
        if (op == OP_CREATE || op == OP_ASSIGN) {
          Var* v = find_or_create(name, nf);
          const bool force = (op == OP_ASSIGN) || (flags & 1);
          std::lock_guard<std::mutex> g(v->mu);
          // the storage of an existing variable is never reallocated: other connection threads
          // hold pointers into it (PULL / PUSH run lock-free); a different size is an error
          if (v->bits.size() != nf) { status |= STATUS_SIZE_MISMATCH; continue; }
          if (!v->init.load() || force) {
            // per-word relaxed atomic stores: concurrent pulls / Hogwild pushes on the same words
            // (a restarted chief re-initialising while non-chiefs train) are not a data race
            const float* src = reinterpret_cast<const float*>(payload.data());
            for (size_t k = 0; k < nf; ++k) st(&v->bits[k], src[k]);
            std::atomic_thread_fence(std::memory_order_release);
            v->init.store(true);
            ++status;
          }
        } else if (op == OP_UNINIT) {
          Var* v = find(name);
          if (!v || !v->init.load()) ++status;
        } else if (op == OP_PULL) {
          Var* v = find(name);
          if (!v || !v->init.load()) { status = 1; snap.emplace_back(); continue; }
          std::vector<uint32_t> s(v->bits.size());
          for (size_t k = 0; k < s.size(); ++k) s[k] = __atomic_load_n(&v->bits[k], __ATOMIC_RELAXED);
          snap.push_back(std::move(s));
          n_pull++;
        } else if (op == OP_PUSH) {
          Var* v = find(name);
          if (!v || v->bits.size() != nf) { status = 2; continue; }
          const float* g = reinterpret_cast<const float*>(payload.data());
          uint32_t* p = v->bits.data();
          if (use_locking) {
            std::lock_guard<std::mutex> lk(v->mu);
            for (size_t k = 0; k < nf; ++k) st(p + k, ld(p + k) - lr * g[k]);
          } else {
            for (size_t k = 0; k < nf; ++k) st(p + k, ld(p + k) - lr * g[k]);
          }
          n_push++;
        } else if (op == OP_INC) {
          Var* v = find(name);
          if (!v || v->bits.empty()) { status = 2; continue; }
          std::lock_guard<std::mutex> lk(v->mu);  // the counter itself is exact
          const float nv = ld(&v->bits[0]) + lr;
          st(&v->bits[0], nv);
          scalar = nv;
        }
      }
      if (!ok) break;
      if (op == OP_PUSH && (flags & 2)) {
        Var* v = find("global_step");
        if (v && !v->bits.empty()) {
          std::lock_guard<std::mutex> lk(v->mu);
          const float nv = ld(&v->bits[0]) + 1.f;
          st(&v->bits[0], nv);
          scalar = nv;
        } else {
          scalar = -1.0;
        }
      }
      if (op == OP_STATS) {
        scalar = (double)n_push.load();
        status = (uint32_t)n_pull.load();
      }
      // respond
      std::string out;
      uint32_t rh[2] = {status, op == OP_PULL ? (uint32_t)snap.size() : 0u};
      out.append(reinterpret_cast<const char*>(rh), 8);
      out.append(reinterpret_cast<const char*>(&scalar), 8);
      if (op == OP_PULL) {
        for (auto& s : snap) {
          uint64_t nb = s.size() * 4;
          out.append(reinterpret_cast<const char*>(&nb), 8);
          out.append(reinterpret_cast<const char*>(s.data()), nb);
          bytes_out += nb;
        }
      }
      if (!write_full(fd, out.data(), out.size())) break;
      if (op == OP_SHUTDOWN) {
        stop.store(true);
        ::shutdown(listen_fd, SHUT_RDWR);
        break;
      }
    }
    ::close(fd);
  }

  void accept_loop() {
    while (!stop.load()) {
      pollfd pfd{listen_fd, POLLIN, 0};
      int pr = ::poll(&pfd, 1, 200);
      if (pr <= 0) continue;
      int fd = ::accept(listen_fd, nullptr, nullptr);
      if (fd < 0) continue;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      std::lock_guard<std::mutex> g(conn_mu);
      conn_fds.push_back(fd);
      conns.emplace_back([this, fd] { handle(fd); });
    }
  }
};

struct Client {
  int fd = -1;
  std::string err;
};

bool send_request(Client* c, uint32_t op, int n, const char** names, const void* const* ptrs, const uint64_t* nbytes,
                  float lr, uint32_t flags, bool with_payload) {
  std::string req;
  uint32_t hdr[5] = {MAGIC, op, (uint32_t)n, 0, flags};
  memcpy(&hdr[3], &lr, 4);
  req.append(reinterpret_cast<const char*>(hdr), sizeof(hdr));
  for (int i = 0; i < n; ++i) {
    uint16_t nl = (uint16_t)strlen(names[i]);
    req.append(reinterpret_cast<const char*>(&nl), 2);
    req.append(names[i], nl);
    uint64_t nb = nbytes ? nbytes[i] : 0;
    req.append(reinterpret_cast<const char*>(&nb), 8);
    if (with_payload && nb) req.append(static_cast<const char*>(ptrs[i]), nb);
  }
  return write_full(c->fd, req.data(), req.size());
}

bool recv_header(Client* c, uint32_t* status, uint32_t* n, double* scalar) {
  uint32_t rh[2];
  if (!read_full(c->fd, rh, 8)) return false;
  if (!read_full(c->fd, scalar, 8)) return false;
  *status = rh[0];
  *n = rh[1];
  return true;
}

}  // namespace

extern "C" {

void* tfx_ps_server_start(const char* host, int port, int use_locking) {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return nullptr;
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  if (!host || !*host || strcmp(host, "0.0.0.0") == 0) {
    addr.sin_addr.s_addr = htonl(INADDR_ANY);  // explicit wildcard only
  } else if (inet_pton(AF_INET, host, &addr.sin_addr) != 1) {
    // a host name: resolve it; never fall back to every interface (the service is unauthenticated)
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host, nullptr, &hints, &res) != 0 || !res) {
      fprintf(stderr, "tfx ps: cannot resolve bind host '%s'\n", host);
      ::close(fd);
      return nullptr;
    }
    addr.sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
    freeaddrinfo(res);
  }
  if (::bind(fd, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0 || ::listen(fd, 64) != 0) {
    ::close(fd);
    return nullptr;
  }
  socklen_t len = sizeof(addr);
  getsockname(fd, reinterpret_cast<sockaddr*>(&addr), &len);
  Server* s = new Server();
  s->listen_fd = fd;
  s->port = ntohs(addr.sin_port);
  s->use_locking = use_locking != 0;
  s->acceptor = std::thread([s] { s->accept_loop(); });
  return s;
}

int tfx_ps_server_port(void* h) { return static_cast<Server*>(h)->port; }
int tfx_ps_server_stopped(void* h) { return static_cast<Server*>(h)->stop.load() ? 1 : 0; }
uint64_t tfx_ps_server_pushes(void* h) { return static_cast<Server*>(h)->n_push.load(); }

void tfx_ps_server_stop(void* h) {
  Server* s = static_cast<Server*>(h);
  s->stop.store(true);
  ::shutdown(s->listen_fd, SHUT_RDWR);
  if (s->acceptor.joinable()) s->acceptor.join();
  {
    std::lock_guard<std::mutex> g(s->conn_mu);
    for (int fd : s->conn_fds) ::shutdown(fd, SHUT_RDWR);
  }
  for (auto& t : s->conns)
    if (t.joinable()) t.join();
  ::close(s->listen_fd);
  delete s;
}

// Copy a variable's current value out of the in-process server (tests / checkpointing on the ps).
int64_t tfx_ps_server_read(void* h, const char* name, float* out, int64_t nfloat) {
  Server* s = static_cast<Server*>(h);
  Var* v = s->find(name);
  if (!v) return -1;
  int64_t n = std::min<int64_t>(nfloat, (int64_t)v->bits.size());
  for (int64_t k = 0; k < n; ++k) out[k] = ld(&v->bits[k]);
  return (int64_t)v->bits.size();
}

void* tfx_ps_connect(const char* host, int port, int timeout_ms) {
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  char ps[16];
  snprintf(ps, sizeof(ps), "%d", port);
  if (getaddrinfo(host, ps, &hints, &res) != 0 || !res) return nullptr;
  int waited = 0;
  while (true) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      freeaddrinfo(res);
      Client* c = new Client();
      c->fd = fd;
      return c;
    }
    if (fd >= 0) ::close(fd);
    if (waited >= timeout_ms) break;
    usleep(50 * 1000);
    waited += 50;
  }
  freeaddrinfo(res);
  return nullptr;
}

void tfx_ps_close(void* h) {
  Client* c = static_cast<Client*>(h);
  if (c->fd >= 0) ::close(c->fd);
  delete c;
}

// returns number of variables (re)initialised by this call, -1 on transport error, -2 if a variable
// already exists on the ps with a different size
int tfx_ps_create(void* h, int n, const char** names, const void* const* ptrs, const uint64_t* nbytes, int force) {
  Client* c = static_cast<Client*>(h);
  if (!send_request(c, OP_CREATE, n, names, ptrs, nbytes, 0.f, force ? 1u : 0u, true)) return -1;
  uint32_t st, k;
  double sc;
  if (!recv_header(c, &st, &k, &sc)) return -1;
  if (st & STATUS_SIZE_MISMATCH) return -2;
  return (int)st;
}

int tfx_ps_uninitialized(void* h, int n, const char** names) {
  Client* c = static_cast<Client*>(h);
  if (!send_request(c, OP_UNINIT, n, names, nullptr, nullptr, 0.f, 0, false)) return -1;
  uint32_t st, k;
  double sc;
  if (!recv_header(c, &st, &k, &sc)) return -1;
  return (int)st;
}

// 0 ok, 1 some variable uninitialised, -1 transport error
int tfx_ps_pull(void* h, int n, const char** names, void* const* ptrs, const uint64_t* nbytes) {
  Client* c = static_cast<Client*>(h);
  if (!send_request(c, OP_PULL, n, names, nullptr, nbytes, 0.f, 0, false)) return -1;
  uint32_t st, k;
  double sc;
  if (!recv_header(c, &st, &k, &sc)) return -1;
  for (uint32_t i = 0; i < k; ++i) {
    uint64_t nb;
    if (!read_full(c->fd, &nb, 8)) return -1;
    if (i < (uint32_t)n && nb == nbytes[i]) {
      if (nb && !read_full(c->fd, ptrs[i], nb)) return -1;
    } else {
      std::vector<char> sink(nb);
      if (nb && !read_full(c->fd, sink.data(), nb)) return -1;
      if (i < (uint32_t)n && nb != nbytes[i]) st = st ? st : 3;
    }
  }
  return (int)st;
}

// apply p -= lr*g on the ps; if inc_step, also global_step += 1 there. *new_step = value after (or -1)
int tfx_ps_push(void* h, int n, const char** names, const void* const* ptrs, const uint64_t* nbytes, float lr,
                int inc_step, double* new_step) {
  Client* c = static_cast<Client*>(h);
  if (!send_request(c, OP_PUSH, n, names, ptrs, nbytes, lr, inc_step ? 2u : 0u, true)) return -1;
  uint32_t st, k;
  double sc;
  if (!recv_header(c, &st, &k, &sc)) return -1;
  if (new_step) *new_step = sc;
  return (int)st;
}

int tfx_ps_inc(void* h, const char* name, float delta, double* value) {
  Client* c = static_cast<Client*>(h);
  const char* names[1] = {name};
  uint64_t nb[1] = {0};
  if (!send_request(c, OP_INC, 1, names, nullptr, nb, delta, 0, false)) return -1;
  uint32_t st, k;
  double sc;
  if (!recv_header(c, &st, &k, &sc)) return -1;
  if (value) *value = sc;
  return (int)st;
}

int tfx_ps_ping(void* h) {
  Client* c = static_cast<Client*>(h);
  if (!send_request(c, OP_PING, 0, nullptr, nullptr, nullptr, 0.f, 0, false)) return -1;
  uint32_t st, k;
  double sc;
  return recv_header(c, &st, &k, &sc) ? 0 : -1;
}

int tfx_ps_shutdown(void* h) {
  Client* c = static_cast<Client*>(h);
  if (!send_request(c, OP_SHUTDOWN, 0, nullptr, nullptr, nullptr, 0.f, 0, false)) return -1;
  uint32_t st, k;
  double sc;
  return recv_header(c, &st, &k, &sc) ? 0 : -1;
}

}  // extern "C"
