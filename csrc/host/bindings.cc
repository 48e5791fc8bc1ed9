// pybind glue for the native host runtime (module paddlebox_amd._pbx_host).
#include <torch/extension.h>

#include "async_dense.h"
#include "cpu_ps.h"
#include "dump.h"
#include "file_mgr.h"
#include "metrics.h"
#include "msg_service.h"
#include "runtime.h"
#include "auc_runner.h"
#include "batch_assembler.h"
#include "tier_store.h"
#include "tier_save.h"
#include "slot_dataset.h"

namespace py = pybind11;
using torch::Tensor;

#define PBX_HOST_CHECK(c, msg) \
  do {                         \
    if (!(c)) throw std::runtime_error(std::string("pbx host: ") + (msg)); \
  } while (0)

namespace pbx {

static void req_cpu(const Tensor& t, const char* n) {
  if (!t.device().is_cpu() || !t.is_contiguous())
    throw std::runtime_error(std::string("pbx host: ") + n + " must be a contiguous CPU tensor");
}

static SparseSGDConfig cfg_from_list(const std::vector<float>& c) {
  SparseSGDConfig s;
  if (c.size() < 16) throw std::runtime_error("sgd config list must have 16 entries");
  s.nonclk_coeff = c[0];
  s.clk_coeff = c[1];
  s.min_bound = c[2];
  s.max_bound = c[3];
  s.learning_rate = c[4];
  s.initial_g2sum = c[5];
  s.initial_range = c[6];
  s.mf_create_thresholds = c[7];
  s.mf_learning_rate = c[8];
  s.mf_initial_g2sum = c[9];
  s.mf_initial_range = c[10];
  s.mf_min_bound = c[11];
  s.mf_max_bound = c[12];
  s.nodeid_slot = c[13];
  s.feature_learning_rate = c[14];
  s.use_feature_lr = (int)c[15];
  return s;
}

static Tensor to_tensor_u64(const std::vector<uint64_t>& v) {
  auto t = torch::empty({(int64_t)v.size()}, torch::kInt64);
  if (!v.empty()) memcpy(t.data_ptr(), v.data(), v.size() * 8);
  return t;
}
static Tensor to_tensor_f(const std::vector<float>& v, int64_t cols) {
  const int64_t rows = cols ? (int64_t)v.size() / cols : 0;
  auto t = torch::empty({rows, cols}, torch::kFloat32);
  if (!v.empty()) memcpy(t.data_ptr(), v.data(), v.size() * 4);
  return t;
}

}  // namespace pbx

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  using namespace pbx;
  register_default_flags();
  m.doc() = "PaddleBox-capability engine: native host runtime";

  // ---------------------------------------------------------------- flags
  m.def("flags_all", [] { return Flags::ins().all(); });
  m.def("flags_help", [] { return Flags::ins().help(); });
  m.def("flag_get", [](const std::string& n) { return Flags::ins().get(n); });
  m.def("flag_set", [](const std::string& n, const std::string& v) { Flags::ins().set(n, v); });
  m.def("flag_define", [](const std::string& n, const std::string& d, const std::string& h) { Flags::ins().define(n, d, h); });

  // ---------------------------------------------------------------- CPU table
  py::class_<SaveFilter>(m, "SaveFilter")
      .def(py::init<>())
      .def_readwrite("base_threshold", &SaveFilter::base_threshold)
      .def_readwrite("delta_threshold", &SaveFilter::delta_threshold)
      .def_readwrite("delta_keep_days", &SaveFilter::delta_keep_days)
      .def_readwrite("embedx_threshold", &SaveFilter::embedx_threshold)
      .def_readwrite("nonclk_coeff", &SaveFilter::nonclk_coeff)
      .def_readwrite("clk_coeff", &SaveFilter::clk_coeff);
  py::class_<CpuTable>(m, "CpuTable")
      .def(py::init<int, int>(), py::arg("dim"), py::arg("nshards") = 16)
      .def_property_readonly("dim", &CpuTable::dim)
      .def_property_readonly("stride", &CpuTable::stride)
      .def("size", &CpuTable::size)
      .def("probe", [](const CpuTable& t, const Tensor& h) {
        req_cpu(h, "h");
        auto rows = torch::empty({h.numel()}, torch::kInt64);
        py::gil_scoped_release nogil;
        t.probe((const uint64_t*)h.data_ptr(), h.numel(), rows.data_ptr<int64_t>());
        return rows;
      })
      .def("insert", [](CpuTable& t, const Tensor& h, float ir, float mir, int init_x, uint64_t seed) {
        req_cpu(h, "h");
        py::gil_scoped_release nogil;
        t.insert((const uint64_t*)h.data_ptr(), h.numel(), ir, mir, init_x != 0, seed);
      })
      .def("gather", [](const CpuTable& t, const Tensor& rows) {
        req_cpu(rows, "rows");
        auto out = torch::empty({rows.numel(), t.stride()}, torch::kFloat32);
        py::gil_scoped_release nogil;
        t.gather(rows.data_ptr<int64_t>(), rows.numel(), out.data_ptr<float>());
        return out;
      })
      .def("assign", [](CpuTable& t, const Tensor& rows, const Tensor& vals) {
        req_cpu(rows, "rows");
        req_cpu(vals, "vals");
        t.assign(rows.data_ptr<int64_t>(), rows.numel(), vals.data_ptr<float>(), (int)vals.size(1));
      })
      .def("push_adagrad", [](CpuTable& t, const Tensor& rows, const Tensor& push, const std::vector<float>& cfg) {
        req_cpu(rows, "rows");
        req_cpu(push, "push");
        auto c = cfg_from_list(cfg);
        static uint64_t seed = 99;
        seed++;
        py::gil_scoped_release nogil;
        t.push_adagrad(rows.data_ptr<int64_t>(), rows.numel(), push.data_ptr<float>(), (int)push.size(1), c, seed);
      })
      .def("shrink", &CpuTable::shrink)
      .def("export_all", [](const CpuTable& t) {
        std::vector<uint64_t> k;
        std::vector<float> v;
        t.export_all(&k, &v);
        return py::make_tuple(to_tensor_u64(k), to_tensor_f(v, t.stride()));
      })
      .def("select_for_save", [](CpuTable& t, int mode, const SaveFilter& f) {
        std::vector<uint64_t> k;
        std::vector<float> v;
        t.select_for_save(mode, f, &k, &v);
        return py::make_tuple(to_tensor_u64(k), to_tensor_f(v, t.stride()));
      })
      .def("erase", [](CpuTable& t, const Tensor& h) {
        req_cpu(h, "h");
        return t.erase((const uint64_t*)h.data_ptr(), h.numel());
      })
      .def("clear", &CpuTable::clear);

  // ---------------------------------------------------------------- metrics
  py::class_<AucCalculator>(m, "AucCalculator")
      .def(py::init<int>(), py::arg("table_size") = 1000000)
      .def("reset", &AucCalculator::reset)
      .def_property_readonly("table_size", &AucCalculator::table_size)
      .def("add", [](AucCalculator& c, const Tensor& pred, const Tensor& label, const c10::optional<Tensor>& mask,
                     float scale) {
        req_cpu(pred, "pred");
        req_cpu(label, "label");
        const float* mk = mask.has_value() ? mask->data_ptr<float>() : nullptr;
        c.add(pred.data_ptr<float>(), label.data_ptr<float>(), mk, pred.numel(), scale);
      }, py::arg("pred"), py::arg("label"), py::arg("mask") = py::none(), py::arg("sample_scale") = 1.0f)
      .def("add_float_label", [](AucCalculator& c, const Tensor& pred, const Tensor& label, const c10::optional<Tensor>& mask) {
        const float* mk = mask.has_value() ? mask->data_ptr<float>() : nullptr;
        c.add_float_label(pred.data_ptr<float>(), label.data_ptr<float>(), mk, pred.numel());
      }, py::arg("pred"), py::arg("label"), py::arg("mask") = py::none())
      .def("add_continue", [](AucCalculator& c, const Tensor& pred, const Tensor& label, const c10::optional<Tensor>& mask) {
        const float* mk = mask.has_value() ? mask->data_ptr<float>() : nullptr;
        c.add_continue(pred.data_ptr<float>(), label.data_ptr<float>(), mk, pred.numel());
      }, py::arg("pred"), py::arg("label"), py::arg("mask") = py::none())
      .def("add_uid", [](AucCalculator& c, const Tensor& pred, const Tensor& label, const Tensor& uid) {
        c.add_uid(pred.data_ptr<float>(), label.data_ptr<float>(), (const uint64_t*)uid.data_ptr(), pred.numel());
      })
      .def("add_nan_inf", [](AucCalculator& c, const Tensor& pred) { c.add_nan_inf(pred.data_ptr<float>(), pred.numel()); })
      .def("merge_tables", [](AucCalculator& c, const Tensor& table, const Tensor& stats) {
        req_cpu(table, "table");
        c.merge_tables(table.data_ptr<double>(), stats.data_ptr<double>());
      })
      .def("tables", [](AucCalculator& c) {
        auto t = torch::empty({2, c.table_size()}, torch::kFloat64);
        memcpy(t.data_ptr<double>(), c.neg().data(), c.table_size() * 8);
        memcpy(t.data_ptr<double>() + c.table_size(), c.pos().data(), c.table_size() * 8);
        auto e = c.local_err();
        auto et = torch::empty({5}, torch::kFloat64);
        memcpy(et.data_ptr<double>(), e.data(), 40);
        return py::make_tuple(t, et);
      })
      .def("compute", [](AucCalculator& c, const c10::optional<Tensor>& tables, const c10::optional<Tensor>& err) {
        if (tables.has_value()) {
          const double* p = tables->data_ptr<double>();
          c.compute(p, p + c.table_size(), err.has_value() ? err->data_ptr<double>() : nullptr);
        } else {
          c.compute_local();
        }
      }, py::arg("tables") = py::none(), py::arg("err") = py::none())
      .def("compute_continue", [](AucCalculator& c, const c10::optional<Tensor>& err) {
        c.compute_continue(err.has_value() ? err->data_ptr<double>() : nullptr);
      }, py::arg("err") = py::none())
      .def("compute_wuauc", &AucCalculator::compute_wuauc)
      .def("compute_nan_inf", &AucCalculator::compute_nan_inf)
      .def_readonly("auc", &AucCalculator::auc)
      .def_readonly("bucket_error", &AucCalculator::bucket_error)
      .def_readonly("mae", &AucCalculator::mae)
      .def_readonly("rmse", &AucCalculator::rmse)
      .def_readonly("actual_ctr", &AucCalculator::actual_ctr)
      .def_readonly("predicted_ctr", &AucCalculator::predicted_ctr)
      .def_readonly("size", &AucCalculator::size)
      .def_readonly("actual_value", &AucCalculator::actual_value)
      .def_readonly("predicted_value", &AucCalculator::predicted_value)
      .def_readonly("uauc", &AucCalculator::uauc)
      .def_readonly("wuauc", &AucCalculator::wuauc)
      .def_readonly("user_cnt", &AucCalculator::user_cnt)
      .def_readonly("nan_cnt", &AucCalculator::nan_cnt)
      .def_readonly("inf_cnt", &AucCalculator::inf_cnt)
      .def_readonly("nan_rate", &AucCalculator::nan_rate)
      .def_readonly("inf_rate", &AucCalculator::inf_rate)
      .def_readonly("nan_inf_rate", &AucCalculator::nan_inf_rate)
      .def_readonly("nan_inf_size", &AucCalculator::nan_inf_size);

  // ---------------------------------------------------------------- dataset
  py::class_<SlotDesc>(m, "SlotDesc")
      .def(py::init<>())
      .def(py::init([](const std::string& name, const std::string& type, bool used, bool dense, int dim) {
             SlotDesc s;
             s.name = name;
             s.type = (type.empty() || type[0] == 'u' || type[0] == 'i') ? 'u' : 'f';
             s.used = used;
             s.dense = dense;
             s.dense_dim = dim;
             return s;
           }),
           py::arg("name"), py::arg("type") = "uint64", py::arg("used") = true, py::arg("dense") = false,
           py::arg("dim") = 1)
      .def_readwrite("name", &SlotDesc::name)
      .def_readwrite("used", &SlotDesc::used)
      .def_readwrite("dense", &SlotDesc::dense)
      .def_readwrite("dense_dim", &SlotDesc::dense_dim);
  py::class_<ParseConfig>(m, "ParseConfig")
      .def(py::init<>())
      .def_readwrite("parse_ins_id", &ParseConfig::parse_ins_id)
      .def_readwrite("parse_logkey", &ParseConfig::parse_logkey)
      .def_readwrite("sample_rate", &ParseConfig::sample_rate)
      .def_readwrite("sample_seed", &ParseConfig::sample_seed);
  py::class_<KeyAgent, std::shared_ptr<KeyAgent>>(m, "KeyAgent")
      .def(py::init<int>(), py::arg("shards") = 64)
      .def("add",
           [](KeyAgent& a, const Tensor& k) {
             req_cpu(k, "keys");
             auto c = k.contiguous().to(torch::kInt64);
             py::gil_scoped_release nogil;
             a.add(reinterpret_cast<const uint64_t*>(c.data_ptr<int64_t>()), (size_t)c.numel());
           })
      .def("keys", [](const KeyAgent& a) { return to_tensor_u64(a.keys()); })
      .def("size", &KeyAgent::size)
      .def("clear", &KeyAgent::clear);
  py::class_<ReplicaStore, std::shared_ptr<ReplicaStore>>(m, "ReplicaStore")
      .def(py::init<int>())
      .def("dim", &ReplicaStore::dim)
      .def("size", &ReplicaStore::size)
      .def("clear", &ReplicaStore::clear)
      .def("add", [](ReplicaStore& r, const Tensor& v) {
        req_cpu(v, "row");
        auto c = v.contiguous().to(torch::kFloat32);
        return r.add(c.data_ptr<float>(), (int)c.numel());
      })
      .def("data", [](const ReplicaStore& r) {
        auto v = r.data();
        auto t = torch::empty({(int64_t)v.size() / r.dim(), r.dim()}, torch::kFloat32);
        if (!v.empty()) memcpy(t.data_ptr(), v.data(), v.size() * 4);
        return t;
      });
  py::class_<InputIndex, std::shared_ptr<InputIndex>>(m, "InputIndex")
      .def(py::init<int>(), py::arg("dim") = 0)
      .def("dim", &InputIndex::dim)
      .def("size", &InputIndex::size)
      .def("add", [](InputIndex& t, const std::string& k, const Tensor& v) {
        req_cpu(v, "vec");
        auto c = v.contiguous().to(torch::kFloat32);
        return t.add(k, c.data_ptr<float>(), (int)c.numel());
      })
      .def("offset", [](const InputIndex& t, const std::string& k) {
        const uint64_t o = t.offset(k.data(), k.size());
        return o == InputIndex::kMissing ? (int64_t)-1 : (int64_t)o;
      })
      .def("load_text", &InputIndex::load_text, py::call_guard<py::gil_scoped_release>())
      .def("data", [](const InputIndex& t) {
        auto v = t.data();
        const int d = std::max(1, t.dim());
        auto o = torch::empty({(int64_t)v.size() / d, d}, torch::kFloat32);
        if (!v.empty()) memcpy(o.data_ptr(), v.data(), v.size() * 4);
        return o;
      });
  py::class_<SlotDataset>(m, "SlotDataset")
      .def(py::init<>())
      .def("set_slots", &SlotDataset::set_slots)
      .def("set_filelist", &SlotDataset::set_filelist)
      .def("set_pipe_command", &SlotDataset::set_pipe_command)
      .def("set_thread_num", &SlotDataset::set_thread_num)
      .def("set_parse", &SlotDataset::set_parse)
      .def("set_so_parser", &SlotDataset::set_so_parser)
      .def("has_so_parser", &SlotDataset::has_so_parser)
      .def("load_into_memory", &SlotDataset::load_into_memory, py::call_guard<py::gil_scoped_release>())
      .def("preload_into_memory", &SlotDataset::preload_into_memory)
      .def("wait_preload_done", &SlotDataset::wait_preload_done, py::call_guard<py::gil_scoped_release>())
      .def("add_lines", &SlotDataset::add_lines)
      .def("release_memory", &SlotDataset::release_memory)
      .def("size", &SlotDataset::size)
      .def("bad_lines", &SlotDataset::bad_lines)
      .def("collect_keys", [](const SlotDataset& d, bool unique) {
        std::vector<uint64_t> k;
        {
          py::gil_scoped_release nogil;
          k = d.collect_keys(unique);
        }
        return to_tensor_u64(k);
      }, py::arg("unique") = true)
      .def("shuffle", &SlotDataset::shuffle)
      .def("set_order", [](SlotDataset& d, const Tensor& o) {
        req_cpu(o, "order");
        std::vector<int64_t> v(o.data_ptr<int64_t>(), o.data_ptr<int64_t>() + o.numel());
        d.set_order(v);
      })
      .def("order", [](const SlotDataset& d) {
        auto& o = d.order();
        auto t = torch::empty({(int64_t)o.size()}, torch::kInt64);
        if (!o.empty()) memcpy(t.data_ptr(), o.data(), o.size() * 8);
        return t;
      })
      .def("set_key_agent", [](SlotDataset& d, std::shared_ptr<KeyAgent> a) { d.set_key_agent(std::move(a)); },
           py::arg("agent").none(true))
      .def("version", &SlotDataset::version)
      .def("set_replica_cache", [](SlotDataset& d, std::shared_ptr<ReplicaStore> r) { d.set_replica_cache(r); },
           py::arg("store").none(true))
      .def("set_input_index", [](SlotDataset& d, std::shared_ptr<InputIndex> t) { d.set_input_index(t); },
           py::arg("table").none(true))
      .def("load_index_files",
           [](const SlotDataset& d, const std::vector<std::string>& files, std::shared_ptr<InputIndex> t) {
             py::gil_scoped_release nogil;
             return d.load_index_files(files, t.get());
           })
      .def("dense_refs", [](const SlotDataset& d) {
        auto v = d.dense_refs();
        auto t = torch::empty({(int64_t)v.size() / 4, 4}, torch::kInt32);
        if (!v.empty()) memcpy(t.data_ptr(), v.data(), v.size() * 4);
        return t;
      })
      // the record store's CSR arrays copied to `device` (u64 values as int64,
      // u64 offsets [nrec*nu+1], f32 values, f32 offsets [nrec*nf+1])
      .def("store_to", [](const SlotDataset& d, const std::string& device) {
        const auto& st = d.store();
        auto dev = torch::Device(device);
        auto copy = [&](const void* p, int64_t n, torch::ScalarType ty) {
          if (n == 0) return torch::empty({0}, torch::TensorOptions().dtype(ty).device(dev));
          auto view = torch::from_blob(const_cast<void*>(p), {n}, torch::TensorOptions().dtype(ty));
          return view.to(dev, /*non_blocking=*/false, /*copy=*/true);
        };
        py::gil_scoped_release nogil;
        return std::make_tuple(copy(st.u64.data(), (int64_t)st.u64.size(), torch::kInt64),
                               copy(st.u64_off.data(), (int64_t)st.u64_off.size(), torch::kInt64),
                               copy(st.f32.data(), (int64_t)st.f32.size(), torch::kFloat32),
                               copy(st.f32_off.data(), (int64_t)st.f32_off.size(), torch::kInt64));
      })
      .def("num_u64_slots", [](const SlotDataset& d) { return d.store().nu; })
      .def("num_f32_slots", [](const SlotDataset& d) { return d.store().nf; })
      .def("merge_by_search_id", [](SlotDataset& d) {
        auto off = d.merge_by_search_id();
        auto t = torch::empty({(int64_t)off.size()}, torch::kInt64);
        memcpy(t.data_ptr(), off.data(), off.size() * 8);
        return t;
      })
      .def("num_sparse_slots", &SlotDataset::num_sparse_slots)
      .def("dense_width", &SlotDataset::dense_width)
      .def("sparse_slot_names", &SlotDataset::sparse_slot_names)
      .def("sparse_slot_u64_index", &SlotDataset::sparse_slot_u64_index)
      .def("dense_slot_names", &SlotDataset::dense_slot_names)
      .def("dense_slot_dims", &SlotDataset::dense_slot_dims)
      .def("build_batch", [](const SlotDataset& d, int64_t begin, int64_t count, bool pin) {
        auto dims = d.batch_dims(begin, count);
        auto opt64 = torch::TensorOptions().dtype(torch::kInt64).pinned_memory(pin);
        auto optf = torch::TensorOptions().dtype(torch::kFloat32).pinned_memory(pin);
        const int S = d.num_sparse_slots();
        auto keys = torch::empty({dims.L}, opt64);
        auto lod = torch::empty({(int64_t)S * (dims.B + 1)}, opt64);
        auto dense = torch::empty({(int64_t)dims.B, d.dense_width()}, optf);
        {
          py::gil_scoped_release nogil;
          d.build_batch(begin, count, keys.data_ptr<int64_t>(), lod.data_ptr<int64_t>(),
                        d.dense_width() ? dense.data_ptr<float>() : nullptr);
        }
        return py::make_tuple(keys, lod, dense);
      }, py::arg("begin"), py::arg("count"), py::arg("pin") = false)
      .def("batch_len", [](const SlotDataset& d, int64_t begin, int64_t count) {
        return d.batch_dims(begin, count).L;
      })
      // fill preallocated (pinned) buffers: keys padded with -1 to keys.numel()
      .def("build_batch_into", [](const SlotDataset& d, int64_t begin, int64_t count, Tensor keys, Tensor lod,
                                  Tensor dense) {
        const int S = d.num_sparse_slots();
        TORCH_CHECK(begin >= 0 && count >= 0 && begin + count <= d.size(), "build_batch_into: range");
        TORCH_CHECK(keys.is_contiguous() && keys.scalar_type() == torch::kInt64, "build_batch_into: keys");
        TORCH_CHECK(lod.is_contiguous() && lod.numel() == (int64_t)S * (count + 1), "build_batch_into: lod");
        TORCH_CHECK(!d.dense_width() || (dense.is_contiguous() && dense.numel() == count * d.dense_width()),
                    "build_batch_into: dense");
        py::gil_scoped_release nogil;
        return d.build_batch_staged(begin, count, keys.data_ptr<int64_t>(), keys.numel(), lod.data_ptr<int64_t>(),
                                    d.dense_width() ? dense.data_ptr<float>() : nullptr);
      })
      .def("build_rank_offset", [](const SlotDataset& d, int64_t begin, int64_t count, int max_rank) {
        auto out = torch::empty({count, 2 * max_rank + 1}, torch::kInt32);
        d.build_rank_offset(begin, count, max_rank, out.data_ptr<int32_t>());
        return out;
      })
      .def("search_ids", [](const SlotDataset& d) { return to_tensor_u64(d.store().search_id); })
      .def("cmatch_rank", [](const SlotDataset& d) {
        const auto& s = d.store();
        auto t = torch::empty({(int64_t)s.cmatch.size()}, torch::kInt64);
        auto* p = t.data_ptr<int64_t>();
        for (size_t i = 0; i < s.cmatch.size(); ++i) p[i] = ((int64_t)s.cmatch[i] << 32) | (int64_t)s.rank[i];
        return t;
      })
      .def("ins_ids", [](const SlotDataset& d) { return d.store().ins_id; })
      .def("batch_ext", [](SlotDataset& d, int64_t begin, int64_t count, int dim) {
        TORCH_CHECK(begin >= 0 && count >= 0 && begin + count <= d.size() && dim > 0, "batch_ext: range");
        auto t = torch::empty({count, dim}, torch::kFloat32);
        d.batch_ext(begin, count, dim, t.data_ptr<float>());
        return t;
      })
      .def("store_ext", [](SlotDataset& d, int64_t begin, int64_t count, int dim, int col, const Tensor& q) {
        TORCH_CHECK(begin >= 0 && count >= 0 && begin + count <= d.size(), "store_ext: range");
        auto qc = q.detach().to(torch::kCPU, torch::kFloat32).contiguous().view(-1);
        TORCH_CHECK(qc.numel() == count, "store_ext: q must hold one value per batch instance");
        d.store_ext(begin, count, dim, col, qc.data_ptr<float>());
      })
      .def("unroll_instances", &SlotDataset::unroll_instances, py::call_guard<py::gil_scoped_release>())
      .def("global_shuffle", &SlotDataset::global_shuffle, py::arg("svc"), py::arg("mode"), py::arg("seed"),
           py::arg("chunk") = 4096, py::arg("threads") = 1, py::call_guard<py::gil_scoped_release>())
      .def("save_archive", &SlotDataset::save_archive)
      .def("load_archive", &SlotDataset::load_archive, py::arg("path"), py::arg("append") = true)
      .def("export_records", [](const SlotDataset& d, const Tensor& idx) {
        // serialise a subset (for the inter-rank shuffle service)
        std::vector<int64_t> v(idx.data_ptr<int64_t>(), idx.data_ptr<int64_t>() + idx.numel());
        RecordStore st = d.store().select(v);
        auto u = to_tensor_u64(st.u64);
        auto uo = torch::from_blob(st.u64_off.data(), {(int64_t)st.u64_off.size()}, torch::kInt64).clone();
        auto f = torch::from_blob(st.f32.data(), {(int64_t)st.f32.size()}, torch::kFloat32).clone();
        auto fo = torch::from_blob(st.f32_off.data(), {(int64_t)st.f32_off.size()}, torch::kInt64).clone();
        auto sid = to_tensor_u64(st.search_id);
        std::vector<int64_t> cr(st.cmatch.size());
        for (size_t i = 0; i < cr.size(); ++i) cr[i] = ((int64_t)st.cmatch[i] << 32) | st.rank[i];
        auto crt = torch::from_blob(cr.data(), {(int64_t)cr.size()}, torch::kInt64).clone();
        return py::make_tuple(u, uo, f, fo, sid, crt);
      })
      .def("import_records", [](SlotDataset& d, const Tensor& u, const Tensor& uo, const Tensor& f, const Tensor& fo,
                                const Tensor& sid, const Tensor& cr) {
        RecordStore st;
        auto& cur = d.mutable_store();
        st.reset(cur.nu, cur.nf);
        st.u64.assign((const uint64_t*)u.data_ptr(), (const uint64_t*)u.data_ptr() + u.numel());
        st.u64_off.assign(uo.data_ptr<int64_t>(), uo.data_ptr<int64_t>() + uo.numel());
        st.f32.assign(f.data_ptr<float>(), f.data_ptr<float>() + f.numel());
        st.f32_off.assign(fo.data_ptr<int64_t>(), fo.data_ptr<int64_t>() + fo.numel());
        st.search_id.assign((const uint64_t*)sid.data_ptr(), (const uint64_t*)sid.data_ptr() + sid.numel());
        for (int64_t i = 0; i < cr.numel(); ++i) {
          st.cmatch.push_back((uint32_t)(cr.data_ptr<int64_t>()[i] >> 32));
          st.rank.push_back((uint32_t)(cr.data_ptr<int64_t>()[i] & 0xffffffff));
        }
        cur.append(st);
        std::vector<int64_t> ord(cur.nrec());
        for (int64_t i = 0; i < (int64_t)ord.size(); ++i) ord[i] = i;
        d.set_order(ord);
        return st.nrec();
      })
      .def("replace_store_with", [](SlotDataset& d, const Tensor& keep) {
        std::vector<int64_t> v(keep.data_ptr<int64_t>(), keep.data_ptr<int64_t>() + keep.numel());
        RecordStore st = d.store().select(v);
        d.mutable_store() = std::move(st);
        std::vector<int64_t> ord(d.store().nrec());
        for (int64_t i = 0; i < (int64_t)ord.size(); ++i) ord[i] = i;
        d.set_order(ord);
      })
      .def("batch_ins_ids", [](const SlotDataset& d, int64_t begin, int64_t count) {
        const auto& o = d.order();
        const auto& ids = d.store().ins_id;
        std::vector<std::string> out((size_t)count);
        for (int64_t i = 0; i < count; ++i) {
          const int64_t r = o.empty() ? begin + i : o[(size_t)(begin + i)];
          if (r >= 0 && r < (int64_t)ids.size()) out[(size_t)i] = ids[(size_t)r];
        }
        return out;
      })
      .def("batch_cmatch_rank", [](const SlotDataset& d, int64_t begin, int64_t count) {
        const auto& o = d.order();
        const auto& s = d.store();
        auto t = torch::zeros({count}, torch::kInt64);
        auto* p = t.data_ptr<int64_t>();
        for (int64_t i = 0; i < count; ++i) {
          const int64_t r = o.empty() ? begin + i : o[(size_t)(begin + i)];
          if (r >= 0 && r < (int64_t)s.cmatch.size()) p[i] = ((int64_t)s.cmatch[(size_t)r] << 32) | s.rank[(size_t)r];
        }
        return t;
      });

  // ---------------------------------------------------------------- file manager
  py::class_<FileMgr, std::unique_ptr<FileMgr, py::nodelete>>(m, "FileMgr")
      .def("init", &FileMgr::init, py::arg("fs_name"), py::arg("fs_ugi"), py::arg("conf_path") = "",
           py::arg("hadoop_bin") = "")
      .def("destroy", &FileMgr::destroy)
      .def_static("is_remote", &FileMgr::is_remote)
      .def("remote_prefix", &FileMgr::remote_prefix)
      .def("list_dir", &FileMgr::list_dir, py::call_guard<py::gil_scoped_release>())
      .def("list_info", &FileMgr::list_info, py::call_guard<py::gil_scoped_release>())
      .def("makedir", &FileMgr::makedir, py::call_guard<py::gil_scoped_release>())
      .def("exists", &FileMgr::exists, py::call_guard<py::gil_scoped_release>())
      .def("download", &FileMgr::download, py::call_guard<py::gil_scoped_release>())
      .def("upload", &FileMgr::upload, py::call_guard<py::gil_scoped_release>())
      .def("remove", &FileMgr::remove, py::call_guard<py::gil_scoped_release>())
      .def("file_size", &FileMgr::file_size, py::call_guard<py::gil_scoped_release>())
      .def("dus", &FileMgr::dus, py::call_guard<py::gil_scoped_release>())
      .def("truncate", &FileMgr::truncate, py::call_guard<py::gil_scoped_release>())
      .def("touch", &FileMgr::touch, py::call_guard<py::gil_scoped_release>())
      .def("rename", &FileMgr::rename, py::call_guard<py::gil_scoped_release>())
      .def("count", &FileMgr::count, py::call_guard<py::gil_scoped_release>())
      .def("last_command", &FileMgr::last_command)
      // whole-file read / write through the same open paths the loaders use
      .def("read_bytes", [](const FileMgr& f, const std::string& path, const std::string& pipe) {
        std::string out;
        {
          py::gil_scoped_release nogil;
          bool is_pipe = false;
          FILE* fp = f.open_read(path, pipe, &is_pipe);
          if (!fp) throw std::runtime_error("cannot open " + path);
          char buf[1 << 16];
          size_t n;
          while ((n = fread(buf, 1, sizeof(buf), fp)) > 0) out.append(buf, n);
          FileMgr::close(fp, is_pipe);
        }
        return py::bytes(out);
      }, py::arg("path"), py::arg("pipe_command") = "")
      .def("write_bytes", [](const FileMgr& f, const std::string& path, const py::bytes& data) {
        std::string d = data;
        py::gil_scoped_release nogil;
        bool is_pipe = false;
        FILE* fp = f.open_write(path, &is_pipe);
        if (!fp) throw std::runtime_error("cannot open for write " + path);
        const bool ok = fwrite(d.data(), 1, d.size(), fp) == d.size();
        FileMgr::close(fp, is_pipe);
        return ok;
      });
  m.def("default_file_mgr", [] { return &default_file_mgr(); }, py::return_value_policy::reference);

  // ---------------------------------------------------------------- shuffle service
  py::class_<MsgService, std::shared_ptr<MsgService>>(m, "MsgService")
      .def(py::init<int, int>(), py::arg("rank"), py::arg("world"))
      .def("listen", &MsgService::listen, py::arg("host"), py::arg("port") = 0)
      .def("connect", &MsgService::connect, py::arg("endpoints"), py::arg("timeout_s") = 60.0,
           py::call_guard<py::gil_scoped_release>())
      .def("register_handler", [](MsgService& s, py::function fn) {
        // the service's threads drop their copies without the GIL: release
        // the Python object under it
        std::shared_ptr<py::function> holder(new py::function(std::move(fn)), [](py::function* f) {
          py::gil_scoped_acquire gil;
          delete f;
        });
        return s.register_handler([holder](int src, const char* buf, int64_t len) {
          py::gil_scoped_acquire gil;
          (*holder)(src, py::bytes(buf ? buf : "", (size_t)len));
        });
      })
      .def("unregister_consumer", &MsgService::unregister_consumer, py::call_guard<py::gil_scoped_release>())
      .def("send_message", [](MsgService& s, int client_id, const py::bytes& data, py::object cb) {
        std::string buf = data;
        MsgService::Callback c;
        if (!cb.is_none()) {
          std::shared_ptr<py::object> holder(new py::object(cb), [](py::object* o) {
            py::gil_scoped_acquire gil;
            delete o;
          });
          c = [holder] {
            py::gil_scoped_acquire gil;
            (*holder)();
          };
        }
        py::gil_scoped_release nogil;
        s.send_message(client_id, buf.data(), (int64_t)buf.size(), std::move(c));
      }, py::arg("client_id"), py::arg("data"), py::arg("callback") = py::none())
      .def("wait_done", &MsgService::wait_done, py::call_guard<py::gil_scoped_release>())
      .def("broken_peers", &MsgService::broken_peers)
      .def("destroy", &MsgService::destroy, py::call_guard<py::gil_scoped_release>())
      .def("bytes_sent", &MsgService::bytes_sent)
      .def("messages_handled", &MsgService::messages_handled)
      .def_property_readonly("rank", &MsgService::rank)
      .def_property_readonly("world", &MsgService::world);

  // ---------------------------------------------------------------- dump
  py::class_<BatchAssembler>(m, "BatchAssembler")
      .def(py::init([](const SlotDataset& ds, py::list jobs, int n_slots) {
             std::vector<BatchAssembler::Job> js;
             for (auto item : jobs) {
               auto t = item.cast<py::tuple>();
               BatchAssembler::Job j;
               j.begin = t[0].cast<int64_t>();
               j.count = t[1].cast<int64_t>();
               Tensor k = t[2].cast<Tensor>(), l = t[3].cast<Tensor>(), d = t[4].cast<Tensor>();
               TORCH_CHECK(k.is_contiguous() && k.scalar_type() == torch::kInt64, "assembler: keys int64");
               TORCH_CHECK(l.is_contiguous() && l.scalar_type() == torch::kInt64 &&
                               l.numel() == (int64_t)ds.num_sparse_slots() * (j.count + 1), "assembler: lod");
               TORCH_CHECK(!ds.dense_width() || (d.is_contiguous() && d.numel() == j.count * ds.dense_width()),
                           "assembler: dense");
               j.keys = k.data_ptr<int64_t>();
               j.keys_cap = k.numel();
               j.lod = l.data_ptr<int64_t>();
               j.dense = ds.dense_width() ? d.data_ptr<float>() : nullptr;
               j.slot = t[5].cast<int>();
               TORCH_CHECK(j.slot < n_slots, "assembler: slot id");
               js.push_back(j);
             }
             return std::make_unique<BatchAssembler>(&ds, std::move(js), n_slots);
           }),
           py::keep_alive<1, 2>())
      .def("start", &BatchAssembler::start)
      .def("next", &BatchAssembler::next, py::call_guard<py::gil_scoped_release>())
      .def("release", &BatchAssembler::release)
      .def("build_seconds", &BatchAssembler::build_seconds)
      .def("wait_seconds", &BatchAssembler::wait_seconds);
  py::class_<HostTier>(m, "HostTier")
      .def(py::init<int, int, int64_t>(), py::arg("stride"), py::arg("threads") = 16,
           py::arg("chunk_rows") = 1 << 20)
      .def("size", &HostTier::size)
      .def("memory_bytes", &HostTier::memory_bytes)
      .def("numa_nodes", &HostTier::numa_nodes)
      .def("stride", &HostTier::stride)
      .def("probe", [](const HostTier& t, const Tensor& h) {
        auto hc = h.contiguous();
        auto rows = torch::empty({hc.numel()}, torch::kInt64);
        {
          py::gil_scoped_release g;
          t.probe(reinterpret_cast<const uint64_t*>(hc.data_ptr<int64_t>()), hc.numel(), rows.data_ptr<int64_t>());
        }
        return rows;
      })
      .def("insert", [](HostTier& t, const Tensor& h) {
        auto hc = h.contiguous();
        auto rows = torch::empty({hc.numel()}, torch::kInt64);
        int64_t fresh = 0;
        {
          py::gil_scoped_release g;
          t.insert(reinterpret_cast<const uint64_t*>(hc.data_ptr<int64_t>()), hc.numel(), rows.data_ptr<int64_t>(),
                   &fresh);
        }
        return py::make_tuple(rows, fresh);
      })
      .def("insert_fresh", [](HostTier& t, const Tensor& h) {
        // (rows, fresh): fresh[i] = h[i] was absent before the call
        auto hc = h.contiguous();
        auto rows = torch::empty({hc.numel()}, torch::kInt64);
        auto fresh = torch::zeros({hc.numel()}, torch::kUInt8);
        {
          py::gil_scoped_release g;
          int64_t n_new = 0;
          t.insert(reinterpret_cast<const uint64_t*>(hc.data_ptr<int64_t>()), hc.numel(), rows.data_ptr<int64_t>(),
                   &n_new, fresh.data_ptr<uint8_t>());
        }
        return py::make_tuple(rows, fresh.to(torch::kBool));
      })
      .def("gather", [](const HostTier& t, const Tensor& rows, Tensor out) {
        TORCH_CHECK(out.is_contiguous() && out.dim() == 2 && out.size(0) >= rows.numel() &&
                    out.scalar_type() == torch::kFloat32, "gather: out [n, stride] f32");
        auto rc = rows.contiguous();
        py::gil_scoped_release g;
        t.gather(rc.data_ptr<int64_t>(), rc.numel(), out.data_ptr<float>(), (int)out.size(1));
      })
      .def("scatter", [](HostTier& t, const Tensor& rows, const Tensor& vals) {
        auto rc = rows.contiguous();
        auto vc = vals.contiguous().to(torch::kFloat32);
        TORCH_CHECK(vc.dim() == 2 && vc.size(0) >= rc.numel(), "scatter: vals");
        py::gil_scoped_release g;
        t.scatter(rc.data_ptr<int64_t>(), rc.numel(), vc.data_ptr<float>(), (int)vc.size(1));
      })
      .def("erase", [](HostTier& t, const Tensor& h) {
        auto hc = h.contiguous();
        py::gil_scoped_release g;  // millions of keys from a write-back thread: the trainer keeps the GIL
        return t.erase(reinterpret_cast<const uint64_t*>(hc.data_ptr<int64_t>()), hc.numel());
      })
      .def("export_all", [](const HostTier& t) {
        std::vector<uint64_t> k;
        std::vector<float> v;
        {
          py::gil_scoped_release g;
          t.export_all(&k, &v);
        }
        return py::make_tuple(to_tensor_u64(k), to_tensor_f(v, t.stride()));
      })
      .def("shrink", &HostTier::shrink, py::arg("decay"), py::arg("unseen_col"), py::arg("nonclk_coeff"),
           py::arg("clk_coeff"), py::arg("delete_threshold"), py::arg("max_unseen"),
           py::call_guard<py::gil_scoped_release>())
      .def("select_ge", [](const HostTier& t, int col, float thr) {
        // the selected rows land straight in the returned tensors (filled by
        // the tier's workers, no intermediate vectors)
        Tensor k, v;
        {
          py::gil_scoped_release g;
          t.select_ge_to(col, thr, [&](size_t n) {
            k = torch::empty({(int64_t)n}, torch::kInt64);
            v = torch::empty({(int64_t)n, (int64_t)t.stride()}, torch::kFloat32);
            return std::make_pair(reinterpret_cast<uint64_t*>(k.data_ptr<int64_t>()), v.data_ptr<float>());
          });
        }
        return py::make_tuple(k, v);
      })
      .def("stamp", [](HostTier& t, const Tensor& rows, int64_t epoch) {
        auto rc = rows.contiguous();
        py::gil_scoped_release g;
        t.stamp(rc.data_ptr<int64_t>(), rc.numel(), (uint32_t)epoch);
      })
      .def("epochs", [](const HostTier& t, const Tensor& rows) {
        auto rc = rows.contiguous();
        auto out = torch::empty({rc.numel()}, torch::kInt64);
        for (int64_t i = 0; i < rc.numel(); ++i) {
          const int64_t r = rc.data_ptr<int64_t>()[i];
          out.data_ptr<int64_t>()[i] = r < 0 ? -1 : (int64_t)t.epoch_of_row(r);
        }
        return out;
      })
      .def("spill_oldest", [](HostTier& t, int64_t keep_rows) {
        Tensor k, v;
        {
          py::gil_scoped_release g;
          t.spill_oldest_to(keep_rows, [&](size_t n) {
            k = torch::empty({(int64_t)n}, torch::kInt64);
            v = torch::empty({(int64_t)n, (int64_t)t.stride()}, torch::kFloat32);
            return std::make_pair(reinterpret_cast<uint64_t*>(k.data_ptr<int64_t>()), v.data_ptr<float>());
          });
        }
        return py::make_tuple(k, v);
      })
      .def("clear", &HostTier::clear);
  py::class_<SsdLog>(m, "SsdLog")
      .def(py::init<const std::string&, int, int64_t>(), py::arg("dir"), py::arg("stride"),
           py::arg("segment_bytes") = 64ll << 20)
      .def("size", &SsdLog::size)
      .def("disk_bytes", &SsdLog::disk_bytes)
      .def("direct_io", &SsdLog::direct_io)
      .def("segments", &SsdLog::segments)
      .def("put", [](SsdLog& s, const Tensor& h, const Tensor& v) {
        auto hc = h.contiguous();
        auto vc = v.contiguous().to(torch::kFloat32);
        TORCH_CHECK(vc.dim() == 2 && vc.size(0) == hc.numel(), "put: one row per key");
        py::gil_scoped_release g;
        s.put(reinterpret_cast<const uint64_t*>(hc.data_ptr<int64_t>()), vc.data_ptr<float>(), hc.numel(),
              (int)vc.size(1));
      })
      .def("get", [](const SsdLog& s, const Tensor& h) {
        auto hc = h.contiguous();
        auto found = torch::zeros({hc.numel()}, torch::kUInt8);
        auto out = torch::empty({hc.numel(), s.stride()}, torch::kFloat32);
        {
          py::gil_scoped_release g;
          s.get(reinterpret_cast<const uint64_t*>(hc.data_ptr<int64_t>()), hc.numel(), found.data_ptr<uint8_t>(),
                out.data_ptr<float>(), s.stride());
        }
        return py::make_tuple(found.to(torch::kBool), out);
      })
      .def("erase", [](SsdLog& s, const Tensor& h) {
        auto hc = h.contiguous();
        py::gil_scoped_release g;
        return s.erase(reinterpret_cast<const uint64_t*>(hc.data_ptr<int64_t>()), hc.numel());
      })
      .def("compact", &SsdLog::compact, py::arg("min_live") = 0.5, py::call_guard<py::gil_scoped_release>())
      .def("shrink", &SsdLog::shrink, py::arg("decay"), py::arg("unseen_col"), py::arg("nonclk_coeff"),
           py::arg("clk_coeff"), py::arg("delete_threshold"), py::arg("max_unseen"),
           py::call_guard<py::gil_scoped_release>())
      .def("live_permille", &SsdLog::live_fraction_permille)
      .def("keys", [](const SsdLog& s) { return to_tensor_u64(s.keys()); });
  m.def(
      "save_tiers",
      [](HostTier* host, SsdLog* ssd, int kind, int mode, bool reset, float base_thr, float delta_thr,
         float keep_days, float nonclk, float clk, float embedx_thr, int dim, const std::string& keys_path,
         const std::string& vals_path, int threads, bool collect) {
        SaveSelect sel;
        sel.mode = mode;
        sel.reset_delta = reset ? 1 : 0;
        sel.base_threshold = base_thr;
        sel.delta_threshold = delta_thr;
        sel.delta_keep_days = keep_days;
        sel.nonclk_coeff = nonclk;
        sel.clk_coeff = clk;
        std::vector<uint64_t> saved;
        TierSaveStats st;
        {
          py::gil_scoped_release g;
          st = save_tiers(host, ssd, kind, sel, dim, embedx_thr, keys_path, vals_path, threads,
                          collect ? &saved : nullptr);
        }
        py::object keys = collect ? py::object(py::cast(to_tensor_u64(saved))) : py::object(py::none());
        return py::make_tuple(st.rows, st.host_rows, st.ssd_rows, st.total_s, keys);
      },
      py::arg("host"), py::arg("ssd"), py::arg("kind"), py::arg("mode"), py::arg("reset"), py::arg("base_threshold"),
      py::arg("delta_threshold"), py::arg("delta_keep_days"), py::arg("nonclk_coeff"), py::arg("clk_coeff"),
      py::arg("embedx_threshold"), py::arg("dim"), py::arg("keys_path"), py::arg("vals_path"), py::arg("threads"),
      py::arg("collect"));
  py::class_<AucRunner>(m, "AucRunner")
      .def(py::init<int, int, uint64_t>(), py::arg("pool_size"), py::arg("threads") = 4, py::arg("seed") = 0)
      .def("set_eval_slots", &AucRunner::set_eval_slots)
      .def("sample", [](AucRunner& a, SlotDataset& d) { a.sample(d.store()); },
           py::call_guard<py::gil_scoped_release>())
      .def("candidate_keys", [](const AucRunner& a) { return to_tensor_u64(a.candidate_keys()); })
      .def("shuffle", [](AucRunner& a, SlotDataset& d, const std::vector<int>& slots) {
             return a.shuffle(&d.mutable_store(), slots);
           }, py::call_guard<py::gil_scoped_release>())
      .def("replaced", &AucRunner::replaced)
      .def("pool_entries", &AucRunner::pool_entries);
  m.def("xxh64", [](const std::string& s, uint64_t seed) { return xxh64(s.data(), s.size(), seed); },
        py::arg("s"), py::arg("seed") = 0);
  py::class_<DumpWriter>(m, "DumpWriter")
      .def(py::init<const std::string&, int, int, size_t>(), py::arg("dir"), py::arg("device_id") = 0,
           py::arg("threads") = 4, py::arg("max_file_len") = (size_t)1 << 31)
      .def("dump_fields", [](DumpWriter& w, const std::vector<std::string>& lineids,
                             const std::vector<std::string>& names, const std::vector<Tensor>& mats, int dump_mode,
                             int dump_interval, bool extend) {
        std::vector<const float*> ptrs;
        std::vector<int64_t> widths;
        int64_t B = (int64_t)lineids.size();
        std::vector<Tensor> keep;
        for (const auto& m0 : mats) {
          auto m1 = m0.to(torch::kCPU).to(torch::kFloat32).contiguous();
          PBX_HOST_CHECK(m1.dim() >= 1 && m1.size(0) == B, "dump field rows != batch size");
          keep.push_back(m1);
          ptrs.push_back(m1.data_ptr<float>());
          widths.push_back(B ? m1.numel() / B : 0);
        }
        py::gil_scoped_release nogil;
        return w.dump_fields(lineids, names, ptrs, widths, B, dump_mode, dump_interval, extend);
      }, py::arg("lineids"), py::arg("names"), py::arg("mats"), py::arg("dump_mode") = 0,
         py::arg("dump_interval") = 1, py::arg("lineid_have_extend_info") = false)
      .def("dump_params", [](DumpWriter& w, int batch_id, const std::vector<std::string>& names,
                             const std::vector<Tensor>& ts) {
        std::vector<const float*> ptrs;
        std::vector<int64_t> lens;
        std::vector<Tensor> keep;
        for (const auto& t0 : ts) {
          auto t1 = t0.to(torch::kCPU).to(torch::kFloat32).contiguous();
          keep.push_back(t1);
          ptrs.push_back(t1.data_ptr<float>());
          lens.push_back(t1.numel());
        }
        py::gil_scoped_release nogil;
        w.dump_params(batch_id, names, ptrs, lens);
      })
      .def("flush", &DumpWriter::flush)
      .def("files", &DumpWriter::files);

  // ---------------------------------------------------------------- async dense table
  py::class_<AsyncDenseTable>(m, "AsyncDenseTable")
      .def(py::init([](const Tensor& params, int64_t adam_len, const Tensor& lr, int device_num, int threads) {
             req_cpu(params, "params");
             req_cpu(lr, "lr");
             auto p = params.to(torch::kFloat32).contiguous();
             auto l = lr.to(torch::kFloat32).contiguous();
             PBX_HOST_CHECK(l.numel() == adam_len, "lr must have adam_len elements");
             return new AsyncDenseTable(p.data_ptr<float>(), p.numel(), adam_len, l.data_ptr<float>(), device_num,
                                        threads);
           }),
           py::arg("params"), py::arg("adam_len"), py::arg("lr"), py::arg("device_num") = 1, py::arg("threads") = 8)
      .def("pull", [](AsyncDenseTable& t, Tensor out) {
        req_cpu(out, "out");
        PBX_HOST_CHECK(out.numel() == t.total_len() && out.is_contiguous(), "pull: bad output");
        py::gil_scoped_release nogil;
        t.pull(out.data_ptr<float>());
      })
      .def("push", [](AsyncDenseTable& t, const Tensor& g) {
        auto g1 = g.to(torch::kCPU).to(torch::kFloat32).contiguous();
        PBX_HOST_CHECK(g1.numel() == t.total_len(), "push: bad gradient length");
        py::gil_scoped_release nogil;
        t.push(g1.data_ptr<float>());
      })
      .def("wait_idle", &AsyncDenseTable::wait_idle, py::call_guard<py::gil_scoped_release>())
      .def("finalize", &AsyncDenseTable::finalize, py::call_guard<py::gil_scoped_release>())
      .def("updates", &AsyncDenseTable::updates)
      .def("total_len", &AsyncDenseTable::total_len)
      .def("snapshot", [](AsyncDenseTable& t, int64_t adam_len) {
        auto p = torch::empty({t.total_len()}, torch::kFloat32);
        auto m = torch::empty({adam_len}, torch::kFloat32);
        auto v = torch::empty({adam_len}, torch::kFloat32);
        t.snapshot(p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>());
        return py::make_tuple(p, m, v);
      });
}
