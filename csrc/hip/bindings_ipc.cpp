// torch glue for the IPC mesh (ipc.hip): memory-handle export / import and
// the collective launches.  Buffers are owned by the Python IpcMesh; this
// side only holds raw pointers and checks sizes.
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include <cstdlib>

#include <cstring>
#include <stdexcept>

#include "kernels.h"

namespace py = pybind11;
using torch::Tensor;

namespace pbx {
namespace {

#define IPC_CHECK(cond, msg)                                                 \
  do {                                                                       \
    if (!(cond)) throw std::runtime_error(std::string("pbx ipc: ") + msg);  \
  } while (0)

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("pbx ipc: ") + what + ": " + hipGetErrorString(e));
}

// (handle bytes, byte offset of t inside its allocation)
py::tuple ipc_handle(const Tensor& t) {
  IPC_CHECK(t.is_cuda(), "tensor must be on the GPU");
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  hip_ok(hipMemGetAddressRange(&base, &size, t.data_ptr()), "hipMemGetAddressRange");
  hipIpcMemHandle_t h;
  hip_ok(hipIpcGetMemHandle(&h, base), "hipIpcGetMemHandle");
  const int64_t off = (int64_t)((char*)t.data_ptr() - (char*)base);
  return py::make_tuple(py::bytes(reinterpret_cast<const char*>(&h), sizeof(h)), off);
}

int64_t ipc_open(const py::bytes& hb, int64_t off) {
  std::string s = hb;
  IPC_CHECK(s.size() == sizeof(hipIpcMemHandle_t), "bad handle size");
  hipIpcMemHandle_t h;
  std::memcpy(&h, s.data(), sizeof(h));
  void* p = nullptr;
  hip_ok(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  return (int64_t)((char*)p + off);
}

void ipc_close(int64_t base) { hip_ok(hipIpcCloseMemHandle(reinterpret_cast<void*>(base)), "hipIpcCloseMemHandle"); }

// Mesh memory that peers write while a kernel of this GPU spins on it:
// hipExtMallocWithFlags(hipDeviceMallocUncached) -- no L2 / MALL caching of
// the lines on any agent, so a peer's xGMI store is visible to a running
// kernel's (system-scope acquire) loads, which HIP guarantees for
// coarse-grained hipMalloc memory only at dispatch / sync boundaries.
// hipDeviceMallocFinegrained (coherent, cacheable) is the other legal choice.
// Zero-filled; freed when the returned tensor dies.
Tensor ipc_buffer(int64_t nbytes, int64_t device, bool uncached) {
  IPC_CHECK(nbytes > 0, "ipc_buffer: size");
  int cur = 0;
  hip_ok(hipGetDevice(&cur), "hipGetDevice");
  hip_ok(hipSetDevice((int)device), "hipSetDevice");
  void* p = nullptr;
  const hipError_t e = hipExtMallocWithFlags(&p, (size_t)nbytes,
                                             uncached ? hipDeviceMallocUncached : hipDeviceMallocFinegrained);
  if (e == hipSuccess) {
    const hipError_t z = hipMemset(p, 0, (size_t)nbytes);
    if (z != hipSuccess) {
      (void)hipFree(p);
      (void)hipSetDevice(cur);
      hip_ok(z, "hipMemset");
    }
  }
  (void)hipSetDevice(cur);
  hip_ok(e, "hipExtMallocWithFlags");
  auto opts = torch::TensorOptions().dtype(torch::kUInt8).device(torch::kCUDA, (int)device);
  return torch::from_blob(p, {nbytes}, [](void* q) { (void)hipFree(q); }, opts);
}

// (memory type, device, allocation flags) of a device pointer: the mesh test
// asserts its buffers are the uncached kind
py::tuple ptr_attrs(int64_t ptr) {
  hipPointerAttribute_t a;
  std::memset(&a, 0, sizeof(a));
  hip_ok(hipPointerGetAttributes(&a, reinterpret_cast<void*>(ptr)), "hipPointerGetAttributes");
  return py::make_tuple((int)a.type, a.device, (int64_t)a.allocationFlags);
}

class IpcComm {
 public:
  // state: own int64 [4] = epoch, arrive|depart (2 x u32), err, pad
  IpcComm(int rank, int world, int64_t slot_bytes, const Tensor& state, int blocks, int depth, int64_t spin_limit)
      : blocks_(blocks) {
    IPC_CHECK(world >= 1 && world <= kIpcMaxRanks && rank >= 0 && rank < world, "rank / world");
    IPC_CHECK(slot_bytes > 0 && slot_bytes % 16 == 0, "slot_bytes must be a positive multiple of 16");
    IPC_CHECK(state.is_cuda() && state.scalar_type() == torch::kInt64 && state.numel() >= 4, "state");
    // power of two: the last block is found by counter % grid, and the
    // 32-bit counters wrap
    IPC_CHECK(blocks >= 1 && blocks <= 1024 && (blocks & (blocks - 1)) == 0, "blocks must be a power of two <= 1024");
    IPC_CHECK(depth >= 2 && depth <= 16, "depth in 2..16");
    IPC_CHECK(spin_limit > 0, "spin_limit");
    std::memset(&p_, 0, sizeof(p_));
    p_.world = world;
    p_.rank = rank;
    p_.depth = depth;
    p_.spin_limit = spin_limit;
    p_.slot_bytes = slot_bytes;
    auto* st = reinterpret_cast<int64_t*>(state.data_ptr());
    p_.epoch = reinterpret_cast<uint64_t*>(st + 0);
    p_.arrive = reinterpret_cast<unsigned int*>(st + 1);
    p_.depart = reinterpret_cast<unsigned int*>(st + 1) + 1;
    p_.err = reinterpret_cast<int*>(st + 2);
    // the per-workgroup system-scope release / acquire stay on: without them
    // (system-coherent inbox accesses alone) the payload self-test failed on
    // a 10 MB, 16-block mesh (profiles/r6_ipc_exchange_bench.txt)
    p_.fence = 1;
  }
  bool fence() const { return p_.fence != 0; }
  void set_peer(int p, int64_t inbox, int64_t flags) {
    IPC_CHECK(p >= 0 && p < p_.world && inbox && flags, "peer");
    p_.inbox[p] = reinterpret_cast<unsigned char*>(inbox);
    p_.flags[p] = reinterpret_cast<uint64_t*>(flags);
  }
  // bound of every later wait (polls of ~55 ns each)
  void set_spin_limit(int64_t v) {
    IPC_CHECK(v > 0, "spin_limit");
    p_.spin_limit = v;
  }
  int64_t spin_limit() const { return p_.spin_limit; }
  void check_ready() const {
    for (int p = 0; p < p_.world; ++p) IPC_CHECK(p_.inbox[p] && p_.flags[p], "peer pointers not set");
  }
  // out = scale * sum over ranks of src (f32, in place allowed).  One-shot up
  // to one slot; two-phase (reduce-scatter + all-gather) needs ceil(n/W)
  // floats per slot.
  void allreduce(const Tensor& src, Tensor out, double scale, bool two_phase) {
    check_ready();
    IPC_CHECK(src.is_cuda() && src.scalar_type() == torch::kFloat32 && src.is_contiguous(), "src");
    IPC_CHECK(out.is_cuda() && out.scalar_type() == torch::kFloat32 && out.is_contiguous() &&
                  out.numel() == src.numel(), "out");
    IPC_CHECK(((uintptr_t)src.data_ptr() & 15) == 0 && ((uintptr_t)out.data_ptr() & 15) == 0,
              "src / out must be 16-byte aligned");
    const int64_t n = src.numel();
    const int W = p_.world;
    if (two_phase) {
      const int64_t cs = ((n + W - 1) / W + 3) / 4 * 4;
      IPC_CHECK(cs * 4 <= p_.slot_bytes, "two-phase chunk larger than the mesh slot");
    } else {
      IPC_CHECK(n * 4 <= p_.slot_bytes, "tensor larger than the mesh slot");
    }
    launch_ipc_allreduce(p_, reinterpret_cast<const float*>(src.data_ptr()),
                         reinterpret_cast<float*>(out.data_ptr()), n, (float)scale, two_phase, blocks_,
                         at::hip::getCurrentHIPStream().stream());
  }
  // all-to-all: send [world, slot_bytes] (contiguous, any dtype) -> dst (same
  // shape); counts / rcounts: optional device int32 [world]
  void exchange(const Tensor& send, Tensor dst, const c10::optional<Tensor>& counts, int64_t rec_bytes,
                bool fill_tail, const c10::optional<Tensor>& rcounts) {
    check_ready();
    IPC_CHECK(send.is_cuda() && send.is_contiguous() && send.nbytes() == (size_t)(p_.world * p_.slot_bytes),
              "send must be contiguous [world, slot_bytes]");
    IPC_CHECK(dst.is_cuda() && dst.is_contiguous() && dst.nbytes() == (size_t)(p_.world * p_.slot_bytes),
              "dst must be contiguous [world, slot_bytes]");
    IPC_CHECK(((uintptr_t)send.data_ptr() & 15) == 0 && ((uintptr_t)dst.data_ptr() & 15) == 0,
              "send / dst must be 16-byte aligned");
    IPC_CHECK(rec_bytes > 0 && rec_bytes <= p_.slot_bytes, "rec_bytes");
    // per-peer record counts travel in the flag word's count field (ipc.hip kIpcCountBits)
    IPC_CHECK(p_.slot_bytes / rec_bytes < ((int64_t)1 << kIpcCountBits),
              "slot holds more records than the flag word's count field can announce");
    const int32_t* c = nullptr;
    int32_t* rc = nullptr;
    if (counts.has_value() && counts->defined()) {
      IPC_CHECK(counts->is_cuda() && counts->scalar_type() == torch::kInt32 && counts->numel() >= p_.world, "counts");
      c = reinterpret_cast<const int32_t*>(counts->data_ptr());
    }
    if (rcounts.has_value() && rcounts->defined()) {
      IPC_CHECK(rcounts->is_cuda() && rcounts->scalar_type() == torch::kInt32 && rcounts->numel() >= p_.world,
                "rcounts");
      rc = reinterpret_cast<int32_t*>(rcounts->data_ptr());
    }
    launch_ipc_exchange(p_, send.data_ptr(), dst.data_ptr(), c, rec_bytes, fill_tail, rc, blocks_,
                        at::hip::getCurrentHIPStream().stream());
  }

  // the mesh's peer table (address, for GpuTable.answer_exchange in the same
  // module) and grid size; the mesh must outlive every launch that uses them
  int64_t peers_ptr() {
    check_ready();
    return (int64_t)reinterpret_cast<uintptr_t>(&p_);
  }
  int blocks() const { return blocks_; }
  // key exchange with the owner pack fused in (launch_ipc_pack_exchange):
  // uniq_h int64 [>= U] (U = u_count[0] on the device), send_index int64,
  // ocnt / rcounts int32 [world] (ocnt zero on entry), overflow int32 [1],
  // dst int64 [world, cap] with cap * 8 <= slot_bytes
  void pack_exchange(const Tensor& uniq_h, const Tensor& u_count, int64_t cap, Tensor send_index, Tensor ocnt,
                     Tensor overflow, Tensor dst, Tensor rcounts) {
    check_ready();
    for (const Tensor* t : std::initializer_list<const Tensor*>{&uniq_h, &u_count, &send_index, &ocnt, &overflow, &dst,
                                                                  &rcounts})
      IPC_CHECK(t->is_cuda() && t->is_contiguous(), "pack_exchange: contiguous device tensors");
    IPC_CHECK(uniq_h.scalar_type() == torch::kInt64 && send_index.scalar_type() == torch::kInt64 &&
                  dst.scalar_type() == torch::kInt64, "pack_exchange: uniq_h / send_index / dst are int64");
    IPC_CHECK(u_count.scalar_type() == torch::kInt32 && ocnt.scalar_type() == torch::kInt32 &&
                  rcounts.scalar_type() == torch::kInt32 && overflow.scalar_type() == torch::kInt32,
              "pack_exchange: counts are int32");
    IPC_CHECK(cap > 0 && cap * 8 <= p_.slot_bytes && cap < ((int64_t)1 << kIpcCountBits), "pack_exchange: cap");
    IPC_CHECK(dst.numel() == (int64_t)p_.world * cap, "pack_exchange: dst must be [world, cap]");
    IPC_CHECK(send_index.numel() >= uniq_h.numel(), "pack_exchange: send_index shorter than uniq_h");
    IPC_CHECK(ocnt.numel() >= p_.world && rcounts.numel() >= p_.world, "pack_exchange: ocnt / rcounts");
    launch_ipc_pack_exchange(p_, reinterpret_cast<const uint64_t*>(uniq_h.data_ptr()),
                             reinterpret_cast<const int32_t*>(u_count.data_ptr()), cap,
                             reinterpret_cast<int64_t*>(send_index.data_ptr()),
                             reinterpret_cast<int32_t*>(ocnt.data_ptr()), reinterpret_cast<int32_t*>(overflow.data_ptr()),
                             reinterpret_cast<uint64_t*>(dst.data_ptr()), reinterpret_cast<int32_t*>(rcounts.data_ptr()),
                             blocks_, at::hip::getCurrentHIPStream().stream());
  }

 private:
  IpcPeers p_;
  int blocks_;
};

}  // namespace

void bind_ipc(py::module& m) {
  m.def("ipc_handle", &ipc_handle);
  m.def("ipc_open", &ipc_open);
  m.def("ipc_close", &ipc_close);
  m.def("ipc_buffer", &ipc_buffer, py::arg("nbytes"), py::arg("device"), py::arg("uncached") = true);
  m.def("ptr_attrs", &ptr_attrs);
  m.attr("kIpcMallocUncached") = (int)hipDeviceMallocUncached;
  m.attr("kIpcMallocFinegrained") = (int)hipDeviceMallocFinegrained;
  py::class_<IpcComm>(m, "IpcComm")
      .def("set_spin_limit", &IpcComm::set_spin_limit)
      .def("spin_limit", &IpcComm::spin_limit)
      .def(py::init<int, int, int64_t, const Tensor&, int, int, int64_t>(), py::arg("rank"), py::arg("world"),
           py::arg("slot_bytes"), py::arg("state"), py::arg("blocks"), py::arg("depth"), py::arg("spin_limit"))
      .def("set_peer", &IpcComm::set_peer)
      .def("allreduce", &IpcComm::allreduce, py::arg("src"), py::arg("out"), py::arg("scale"),
           py::arg("two_phase"))
      .def("exchange", &IpcComm::exchange, py::arg("send"), py::arg("dst"), py::arg("counts"), py::arg("rec_bytes"),
           py::arg("fill_tail"), py::arg("rcounts"))
      .def("pack_exchange", &IpcComm::pack_exchange)
      .def("peers_ptr", &IpcComm::peers_ptr)
      .def("blocks", &IpcComm::blocks)
      .def("fence", &IpcComm::fence);
}

}  // namespace pbx
