// pybind11 / torch binding of the shared-memory step-plan ring (core: step_ring.h).
#include "step_ring.h"

#include <pybind11/pybind11.h>
#include <torch/extension.h>

namespace vgate {

class StepRing {
 public:
  StepRing(const std::string& name, bool create, int64_t slots, int64_t slot_bytes, int64_t followers)
      : core_(name, create, slots, slot_bytes, followers) {}

  bool publish(int64_t T, int64_t S, int64_t ns, int64_t nt, int64_t mode, const torch::Tensor& data,
               int64_t nbytes, double timeout_s) {
    TORCH_CHECK(!data.is_cuda() && data.is_contiguous() && data.scalar_type() == torch::kUInt8,
                "StepRing.publish: contiguous uint8 CPU tensor");
    TORCH_CHECK(nbytes >= 0 && nbytes <= data.numel() && nbytes <= core_.slot_bytes(),
                "StepRing.publish: payload larger than a slot");
    pybind11::gil_scoped_release nogil;
    return core_.publish(T, S, ns, nt, mode, data.data_ptr(), (size_t)nbytes, timeout_s);
  }

  pybind11::tuple wait(int64_t f, torch::Tensor& out, double timeout_s) {
    TORCH_CHECK(!out.is_cuda() && out.is_contiguous() && out.scalar_type() == torch::kUInt8,
                "StepRing.wait: contiguous uint8 CPU tensor");
    StepRingCore::Step st;
    {
      pybind11::gil_scoped_release nogil;
      st = core_.wait(f, out.data_ptr(), (size_t)out.numel(), timeout_s);
    }
    return pybind11::make_tuple(st.T, st.S, st.ns, st.nt, st.mode, st.nbytes);
  }

  StepRingCore& core() { return core_; }

 private:
  StepRingCore core_;
};

void bind_step_ring(pybind11::module_& m) {
  namespace py = pybind11;
  py::class_<StepRing>(m, "StepRing", "shared-memory step-plan ring: TP rank 0 -> follower ranks")
      .def(py::init<const std::string&, bool, int64_t, int64_t, int64_t>(), py::arg("name"), py::arg("create"),
           py::arg("slots") = 8, py::arg("slot_bytes") = 1 << 20, py::arg("followers") = 1)
      .def("publish", &StepRing::publish, py::arg("T"), py::arg("S"), py::arg("ns"), py::arg("nt"), py::arg("mode"),
           py::arg("data"), py::arg("nbytes"), py::arg("timeout_s") = 0.0)
      .def("wait", &StepRing::wait, py::arg("follower"), py::arg("out"), py::arg("timeout_s") = 0.0)
      .def("heartbeat", [](StepRing& r) { r.core().heartbeat(); })
      .def("close", [](StepRing& r) { r.core().close_ring(); })
      .def("unlink", [](StepRing& r) { r.core().unlink(); })
      .def("published", [](StepRing& r) { return r.core().published(); })
      .def("acked", [](StepRing& r, int64_t f) { return r.core().acked(f); })
      .def_property_readonly("slots", [](StepRing& r) { return r.core().slots(); })
      .def_property_readonly("slot_bytes", [](StepRing& r) { return r.core().slot_bytes(); })
      .def_property_readonly("name", [](StepRing& r) { return r.core().name(); });
}

}  // namespace vgate
