// Sanitizer stress driver for the host runtime (SURVEY.md §5.2 race detection, test tier
// T-sanitize).  Built by tests/test_runtime_sanitizers.py twice -- -fsanitize=thread and
// -fsanitize=address,undefined -- straight from csrc/runtime/*.cpp, and run on the CPU:
//
//  * parameter-server service: an in-process server, NCLIENT client threads doing the async
//    worker loop (create-if-absent, pull, Hogwild push with global-step increment, counter inc)
//    concurrently -- the reference's lock-free ApplyGradientDescent from several workers
//    (R/distributed/distributed.py:108) -- then an exact global-step check and a clean shutdown
//    while connections are open;
//  * tfevents writer: scalar records from one producer while the background flush thread drains,
//    explicit flushes racing it, then close.
//
// Exit code 0 = every check passed; the sanitizers abort the process on a finding.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* tfx_ps_server_start(const char* host, int port, int use_locking);
int tfx_ps_server_port(void* h);
void tfx_ps_server_stop(void* h);
int64_t tfx_ps_server_read(void* h, const char* name, float* out, int64_t nfloat);
void* tfx_ps_connect(const char* host, int port, int timeout_ms);
void tfx_ps_close(void* h);
int tfx_ps_create(void* h, int n, const char** names, const void* const* ptrs, const uint64_t* nbytes, int force);
int tfx_ps_pull(void* h, int n, const char** names, void* const* ptrs, const uint64_t* nbytes);
int tfx_ps_push(void* h, int n, const char** names, const void* const* ptrs, const uint64_t* nbytes, float lr,
                int inc_step, double* new_step);
int tfx_ps_inc(void* h, const char* name, float delta, double* value);
void* tfx_events_open(const char* path, double wall_time);
void tfx_events_add_scalars(void* h, int64_t step, double wall_time, int n, const char** tags, const float* vals);
void tfx_events_flush(void* h);
uint64_t tfx_events_written(void* h);
void tfx_events_close(void* h);
}

#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                      \
    }                                                               \
  } while (0)

static int ps_stress(int nclient, int steps, int use_locking) {
  void* srv = tfx_ps_server_start("127.0.0.1", 0, use_locking);
  CHECK(srv != nullptr);
  const int port = tfx_ps_server_port(srv);
  const char* names[3] = {"global_step", "weights/Variable", "biases/Variable"};
  const uint64_t nb[3] = {4, 784 * 100 * 4, 100 * 4};
  std::vector<std::thread> th;
  for (int w = 0; w < nclient; ++w) {
    th.emplace_back([&, w] {
      void* c = tfx_ps_connect("127.0.0.1", port, 5000);
      CHECK(c != nullptr);
      std::vector<float> step(1, 0.f), W(784 * 100, 0.5f), b(100, 0.f), g(784 * 100, 1e-3f), gb(100, 1e-3f);
      const void* init[3] = {step.data(), W.data(), b.data()};
      CHECK(tfx_ps_create(c, 3, names, init, nb, 0) >= 0);  // chief-or-not: create if absent
      void* out[3] = {step.data(), W.data(), b.data()};
      const void* grads[2] = {g.data(), gb.data()};
      for (int s = 0; s < steps; ++s) {
        CHECK(tfx_ps_pull(c, 3, names, out, nb) == 0);
        double ns = -1;
        CHECK(tfx_ps_push(c, 2, names + 1, grads, nb + 1, 0.01f, 1, &ns) == 0);
        CHECK(ns >= 1.0);
      }
      double v = 0;
      CHECK(tfx_ps_inc(c, "global_step", 0.f, &v) == 0);
      (void)w;
      tfx_ps_close(c);
    });
  }
  // a restarted chief re-initialising (force) while the workers pull and push
  th.emplace_back([&] {
    void* c = tfx_ps_connect("127.0.0.1", port, 5000);
    CHECK(c != nullptr);
    std::vector<float> W(784 * 100, 0.25f), b(100, 0.f);
    const void* init[2] = {W.data(), b.data()};
    for (int s = 0; s < steps / 10 + 1; ++s) CHECK(tfx_ps_create(c, 2, names + 1, init, nb + 1, 1) >= 0);
    // a size mismatch on an existing variable is rejected, never reallocated
    const uint64_t bad[1] = {8};
    CHECK(tfx_ps_create(c, 1, names + 2, init + 1, bad, 1) == -2);
    tfx_ps_close(c);
  });
  for (auto& t : th) t.join();
  float gs = -1.f;
  CHECK(tfx_ps_server_read(srv, "global_step", &gs, 1) == 1);
  if ((int)gs != nclient * steps) {
    fprintf(stderr, "global_step %f != %d\n", gs, nclient * steps);
    return 1;
  }
  // stop with a client still connected: the server must shut its connection threads down cleanly
  void* idle = tfx_ps_connect("127.0.0.1", port, 5000);
  CHECK(idle != nullptr);
  tfx_ps_server_stop(srv);
  tfx_ps_close(idle);
  return 0;
}

static int events_stress(const char* dir, int records) {
  std::string path = std::string(dir) + "/events.out.tfevents.stress";
  void* h = tfx_events_open(path.c_str(), 1.0);
  CHECK(h != nullptr);
  const char* tags[2] = {"cost", "accuracy"};
  std::thread flusher([&] {
    for (int i = 0; i < 50; ++i) tfx_events_flush(h);
  });
  for (int i = 0; i < records; ++i) {
    const float vals[2] = {1.f / (i + 1), (float)i / records};
    tfx_events_add_scalars(h, i, 1.0 + i, 2, tags, vals);
  }
  flusher.join();
  tfx_events_flush(h);
  CHECK(tfx_events_written(h) >= (uint64_t)records);
  tfx_events_close(h);
  FILE* f = fopen(path.c_str(), "rb");
  CHECK(f != nullptr);
  fseek(f, 0, SEEK_END);
  const long sz = ftell(f);
  fclose(f);
  CHECK(sz > records * 16);
  return 0;
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp";
  int rc = ps_stress(4, 200, 0);
  rc |= ps_stress(3, 100, 1);
  rc |= events_stress(dir, 2000);
  if (rc == 0) printf("RT_STRESS_OK\n");
  return rc;
}
