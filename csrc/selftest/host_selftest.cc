// Standalone self-test of the native host runtime (no Python, no torch), built
// under ASan+UBSan and TSan by scripts/sanitize_host.sh (the
// reference only offers SANITIZER_TYPE build flags; here every sanitizer build
// runs this driver).  It drives the concurrent paths: the multi-threaded pass
// loader (built-in parser and a dlopen'ed plugin), the async dense table
// (concurrent pushers vs. the update thread vs. pullers), the dump writer
// threads, the shuffle message service (3 in-process ranks shuffling their
// datasets over the TCP mesh at once), plus the CPU sparse table and the AUC
// calculator.
//
//   host_selftest <workdir> [plugin.so]
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "host/async_dense.h"
#include "host/cpu_ps.h"
#include "host/dump.h"
#include "host/metrics.h"
#include "host/msg_service.h"
#include "host/slot_dataset.h"

using namespace pbx;

static int g_fail = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                       \
    }                                                                 \
  } while (0)

static std::vector<SlotDesc> slots() {
  std::vector<SlotDesc> s(3);
  s[0].name = "label"; s[0].type = 'u'; s[0].dense = true; s[0].dense_dim = 1;
  s[1].name = "s1"; s[1].type = 'u';
  s[2].name = "s2"; s[2].type = 'u';
  return s;
}

static void test_dataset(const std::string& dir) {
  std::vector<std::string> files;
  for (int f = 0; f < 6; ++f) {
    const std::string p = dir + "/part-" + std::to_string(f);
    std::ofstream o(p);
    for (int i = 0; i < 500; ++i) o << "1 " << (i & 1) << " 2 " << (f * 1000 + i + 1) << " " << (i + 7) << " 1 " << (i % 13 + 1) << "\n";
    files.push_back(p);
  }
  SlotDataset d;
  d.set_slots(slots());
  d.set_thread_num(4);
  d.set_filelist(files);
  // loader threads register feasigns into the feed-pass agent concurrently
  auto agent = std::make_shared<KeyAgent>(16);
  d.set_key_agent(agent);
  CHECK(d.load_into_memory() == 3000);
  d.preload_into_memory();  // second pass on a background thread
  CHECK(d.wait_preload_done() == 6000);
  d.set_key_agent(nullptr);
  CHECK(agent->size() == 3006);
  d.shuffle(7);
  auto dims = d.batch_dims(0, 64);
  std::vector<int64_t> keys(dims.L), lod(2 * 65);
  std::vector<float> dense(64 * d.dense_width());
  d.build_batch(0, 64, keys.data(), lod.data(), dense.data());
  CHECK(dims.L == 64 * 3);
  std::vector<int64_t> keys2(dims.L + 5), lod2(2 * 65);
  std::vector<float> dense2(64 * d.dense_width());
  CHECK(d.build_batch_staged(0, 64, keys2.data(), (int64_t)keys2.size(), lod2.data(), dense2.data()) == dims.L);
  CHECK(std::equal(keys.begin(), keys.end(), keys2.begin()) && keys2[dims.L] == -1 && lod == lod2);
  CHECK(d.collect_keys(true).size() == 3006);  // s1: 3000 ids; s2/s3 add 501..506
  d.save_archive(dir + "/arch");
  SlotDataset e;
  e.set_slots(slots());
  CHECK(e.load_archive(dir + "/arch", false) == 6000);
}

static void test_plugin(const std::string& dir, const char* so) {
  std::vector<SlotDesc> s(3);
  s[0].name = "label"; s[0].type = 'u'; s[0].dense = true;
  s[1].name = "C1"; s[1].type = 'u';
  s[2].name = "C2"; s[2].type = 'u';
  const std::string p = dir + "/criteo.tsv";
  {
    std::ofstream o(p);
    for (int i = 0; i < 2000; ++i) {
      o << (i & 1);
      for (int k = 0; k < 13; ++k) o << "\t" << i;
      for (int k = 0; k < 26; ++k) o << "\t" << std::hex << (0x100 + i % 50) << std::dec;
      o << "\n";
    }
  }
  SlotDataset d;
  d.set_slots(s);
  d.set_so_parser(so);
  d.set_thread_num(4);
  d.set_filelist({p, p, p});
  CHECK(d.load_into_memory() == 6000);
  CHECK(d.collect_keys(true).size() == 100);
}

static void test_async_dense() {
  const int64_t T = 4096;
  std::vector<float> p(T, 0.5f), lr(T, 0.01f);
  AsyncDenseTable t(p.data(), T, T, lr.data(), 4, 4);
  std::vector<std::thread> th;
  std::atomic<int> pulls{0};
  for (int w = 0; w < 4; ++w)
    th.emplace_back([&, w] {
      std::vector<float> g(T, 0.1f * (w + 1)), out(T);
      for (int it = 0; it < 50; ++it) {
        t.pull(out.data());
        t.push(g.data());
        ++pulls;
      }
    });
  for (auto& x : th) x.join();
  t.wait_idle();
  CHECK(t.updates() > 0);
  std::vector<float> out(T);
  t.pull(out.data());
  CHECK(out[0] < 0.5f && std::isfinite(out[T - 1]));
  t.finalize();
}

static void test_dump(const std::string& dir) {
  DumpWriter w(dir + "/dump", 0, 4, 4096);
  std::vector<std::string> ids;
  std::vector<float> a(200 * 3);
  for (int i = 0; i < 200; ++i) ids.push_back("line" + std::to_string(i));
  for (size_t i = 0; i < a.size(); ++i) a[i] = (float)i;
  std::vector<std::thread> th;
  for (int k = 0; k < 4; ++k)
    th.emplace_back([&] { w.dump_fields(ids, {"f"}, {a.data()}, {3}, 200, 0, 1, false); });
  for (auto& x : th) x.join();
  w.flush();
  CHECK(!w.files().empty());
}

static void test_cpu_table_and_auc() {
  CpuTable t(8, 16);
  std::vector<uint64_t> h(10000);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (i * 0x9E3779B97F4A7C15ULL) | 1;
  t.insert(h.data(), (int64_t)h.size(), 0.f, 1e-4f, true, 1);
  CHECK(t.size() == 10000);
  std::vector<int64_t> rows(h.size());
  t.probe(h.data(), (int64_t)h.size(), rows.data());
  for (auto r : rows) CHECK(r >= 0);
  std::vector<float> v(h.size() * t.stride());
  t.gather(rows.data(), (int64_t)rows.size(), v.data());
  t.assign(rows.data(), (int64_t)rows.size(), v.data(), t.stride());
  CHECK(t.erase(h.data(), 100) == 100);
  CHECK(t.size() == 9900);

  AucCalculator c(1000);
  std::vector<float> pred(4000), label(4000);
  for (int i = 0; i < 4000; ++i) {
    label[i] = (float)(i & 1);
    pred[i] = label[i] > 0 ? 0.6f + 0.0001f * (i % 100) : 0.4f - 0.0001f * (i % 100);
  }
  c.add(pred.data(), label.data(), nullptr, 4000);
  c.compute_local();
}

static void test_global_shuffle() {
  const int W = 3;
  std::vector<std::unique_ptr<MsgService>> svc;
  std::vector<std::string> eps;
  for (int r = 0; r < W; ++r) {
    svc.emplace_back(new MsgService(r, W));
    eps.push_back("127.0.0.1:" + std::to_string(svc[r]->listen("127.0.0.1", 0)));
  }
  std::vector<std::unique_ptr<SlotDataset>> ds;
  std::vector<std::string> lines;
  for (int r = 0; r < W; ++r) {
    ds.emplace_back(new SlotDataset());
    ds[r]->set_slots(slots());
    lines.clear();
    for (int i = 0; i < 300 + 50 * r; ++i)
      lines.push_back("1 " + std::to_string(i & 1) + " 1 " + std::to_string(r * 10000 + i + 1) + " 1 999999");
    ds[r]->add_lines(lines);
  }
  std::vector<std::thread> ts;
  std::atomic<int64_t> moved{0};
  for (int r = 0; r < W; ++r)
    ts.emplace_back([&, r] {
      svc[r]->connect(eps);
      moved += ds[r]->global_shuffle(*svc[r], 0, 11, 23, 2);
    });
  for (auto& t : ts) t.join();
  int64_t total = 0;
  std::vector<uint64_t> all;
  for (int r = 0; r < W; ++r) {
    total += ds[r]->size();
    auto k = ds[r]->collect_keys(false);
    all.insert(all.end(), k.begin(), k.end());
  }
  CHECK(total == 300 + 350 + 400);
  CHECK(moved.load() > 0);
  std::sort(all.begin(), all.end());
  all.erase(std::unique(all.begin(), all.end()), all.end());
  CHECK(all.size() == (size_t)total + 1);  // every s1 id once, plus the shared s2 feasign
  for (auto& s : svc) s->destroy();
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: host_selftest <workdir> [plugin.so]\n");
    return 2;
  }
  const std::string dir = argv[1];
  test_dataset(dir);
  if (argc > 2) test_plugin(dir, argv[2]);
  test_async_dense();
  test_dump(dir);
  test_cpu_table_and_auc();
  test_global_shuffle();
  if (g_fail) {
    fprintf(stderr, "host_selftest: %d check(s) failed\n", g_fail);
    return 1;
  }
  printf("host_selftest: ok\n");
  return 0;
}
