// py_e2sar.cpp -- the e2sar_py module surface for the MI355X SAR path.
//
// Same module layout and names as the reference bindings (src/pybind/py_e2sar.cpp,
// py_e2sarDP.cpp, py_e2sarHeaders.cpp): E2SARErrorc / E2SARErrorInfo / result types,
// EjfatURI, IPAddress, the header classes, and the DataPlane submodule with
// Segmenter / Reassembler and their bytes / buffer / numpy methods, including the
// (len | -1 empty | -2 error, data, eventNum, dataId) return convention.
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "e2sar_amd/e2sar.hpp"
#include "e2sar_amd/e2sarHeaders.hpp"

namespace py = pybind11;
using namespace e2sar;

namespace {

template <typename T>
void bind_result(py::module_ &m, const char *name)
{
    py::class_<result<T>>(m, name)
        .def("value", [](const result<T> &r) { return r.value(); })
        .def("error", [](const result<T> &r) -> E2SARErrorInfo {
            if (r.has_error()) return r.error();
            throw std::runtime_error("No error present in result");
        })
        .def("has_error", [](const result<T> &r) { return r.has_error(); })
        .def("has_value", [](const result<T> &r) { return r.has_value(); });
}

struct IPAddress {
    std::string s;
};

enum class TokenType { admin = 0, instance = 1, session = 2 };   // EjfatURI::TokenType

// Python callbacks from the send thread: re-acquire the GIL (py_e2sarDP.cpp:36-79)
struct PyCallback {
    py::object cb, arg;
    static void execute(std::any a)
    {
        auto *w = std::any_cast<PyCallback *>(a);
        {
            py::gil_scoped_acquire gil;
            try {
                w->cb(w->arg);
            } catch (py::error_already_set &e) {
                PyErr_Print();
            }
            w->cb = py::object();
            w->arg = py::object();
        }
        delete w;
    }
};

py::tuple event_tuple_bytes(result<int> r, uint8_t *buf, size_t len, EventNum_t ev, uint16_t did)
{
    if (r.has_error()) return py::make_tuple(-2, py::bytes(), ev, did);
    if (r.value() == -1 || buf == nullptr) return py::make_tuple(-1, py::bytes(), ev, did);
    py::bytes b(reinterpret_cast<const char *>(buf), len);
    delete[] buf;
    return py::make_tuple(len, b, ev, did);
}

py::tuple event_tuple_array(result<int> r, uint8_t *buf, size_t len, EventNum_t ev, uint16_t did, py::dtype dt)
{
    if (r.has_error()) return py::make_tuple(-2, py::array(), ev, did);
    if (r.value() == -1) return py::make_tuple(-1, py::array(), ev, did);
    const py::ssize_t n = static_cast<py::ssize_t>(len) / dt.itemsize();
    py::capsule owner(buf, [](void *p) { delete[] static_cast<uint8_t *>(p); });
    return py::make_tuple(len, py::array(dt, {n}, buf, owner), ev, did);
}

}  // namespace

PYBIND11_MODULE(e2sar_py, m)
{
    m.doc() = "E2SAR data-plane SAR on MI355X (gfx950): reference-shaped Python API";
    py::register_exception<E2SARException>(m, "E2SARException");
    m.attr("_dp_port") = py::int_(DATAPLANE_PORT);
    m.attr("_iphdr_len") = py::int_(IP_HDRLEN);
    m.attr("_udphdr_len") = py::int_(UDP_HDRLEN);
    m.attr("_total_hdr_len") = py::int_(TOTAL_HDR_LEN);
    m.attr("_rehdr_version_nibble") = py::int_(rehdrVersionNibble);
    m.def("get_version", []() { return std::string("0.3.2-mi355x"); });
    m.def("_get_PortRange", &get_PortRange, py::arg("source_count"));   // e2sarCP.hpp:772-798

    py::enum_<E2SARErrorc>(m, "E2SARErrorc")
        .value("NoError", E2SARErrorc::NoError)
        .value("CaughtException", E2SARErrorc::CaughtException)
        .value("ParseError", E2SARErrorc::ParseError)
        .value("ParameterError", E2SARErrorc::ParameterError)
        .value("ParameterNotAvailable", E2SARErrorc::ParameterNotAvailable)
        .value("OutOfRange", E2SARErrorc::OutOfRange)
        .value("Undefined", E2SARErrorc::Undefined)
        .value("NotFound", E2SARErrorc::NotFound)
        .value("RPCError", E2SARErrorc::RPCError)
        .value("SocketError", E2SARErrorc::SocketError)
        .value("MemoryError", E2SARErrorc::MemoryError)
        .value("LogicError", E2SARErrorc::LogicError)
        .value("SystemError", E2SARErrorc::SystemError)
        .value("DataError", E2SARErrorc::DataError)
        .export_values();

    py::class_<E2SARErrorInfo>(m, "E2SARErrorInfo")
        .def_property_readonly("code", &E2SARErrorInfo::code)
        .def_property_readonly("message", &E2SARErrorInfo::message)
        .def("__repr__", [](const E2SARErrorInfo &e) {
            return "<E2SARErrorInfo(code=" + std::to_string(static_cast<int>(e.code())) + ", message='" + e.message() +
                   "')>";
        });

    bind_result<int>(m, "E2SARResultInt");
    bind_result<SegmenterFlagsT>(m, "E2SARResultSegmenterFlags");
    bind_result<ReassemblerFlagsT>(m, "E2SARResultReassemblerFlags");
    bind_result<std::list<std::pair<uint16_t, size_t>>>(m, "E2SARResultListOfFDPairs");

    py::class_<IPAddress>(m, "IPAddress")
        .def(py::init<>())
        .def_static("from_string", [](const std::string &s) { return IPAddress{s}; })
        .def("is_v4", [](const IPAddress &a) { return a.s.find(':') == std::string::npos; })
        .def("is_v6", [](const IPAddress &a) { return a.s.find(':') != std::string::npos; })
        .def("__str__", [](const IPAddress &a) { return a.s; });

    py::class_<EjfatURI> uri(m, "EjfatURI");
    py::enum_<TokenType>(uri, "TokenType")
        .value("admin", TokenType::admin)
        .value("instance", TokenType::instance)
        .value("session", TokenType::session);
    uri.def(py::init([](const std::string &u, TokenType, bool) { return EjfatURI(u); }), py::arg("uri"),
            py::arg("tt") = TokenType::admin, py::arg("preferV6") = false)
        .def("has_data_addr_v4", &EjfatURI::has_dataAddrv4)
        .def("has_data_addr_v6", &EjfatURI::has_dataAddrv6)
        .def("has_data_addr", &EjfatURI::has_dataAddr)
        .def("has_sync_addr", &EjfatURI::has_syncAddr)
        .def("get_lb_id", &EjfatURI::get_lbId);

    // ---- headers (py_e2sarHeaders.cpp) ----
    py::class_<REHdr>(m, "REHdr")
        .def(py::init<>())
        .def("set", &REHdr::set, py::arg("data_id") = 0, py::arg("buff_off") = 0, py::arg("buff_len") = 0,
             py::arg("event_num") = 0)
        .def("get_eventNum", &REHdr::get_eventNum)
        .def("get_bufferLength", &REHdr::get_bufferLength)
        .def("get_bufferOffset", &REHdr::get_bufferOffset)
        .def("get_dataId", &REHdr::get_dataId)
        .def("get_headerVersion", &REHdr::get_HeaderVersion)
        .def("validate", &REHdr::validate)
        .def("get_fields", &REHdr::get_Fields)
        .def("to_bytes", [](const REHdr &h) { return py::bytes(reinterpret_cast<const char *>(&h), sizeof(h)); })
        .def_static("from_bytes", [](py::bytes b) {
            std::string s = b;
            if (s.size() < sizeof(REHdr)) throw std::invalid_argument("need 20 bytes");
            REHdr h;
            std::memcpy(static_cast<void *>(&h), s.data(), sizeof(REHdr));
            return h;
        });
    py::class_<LBHdrV2>(m, "LBHdrV2")
        .def(py::init<>())
        .def("set", &LBHdrV2::set, py::arg("entropy") = 0, py::arg("event_num") = 0)
        .def("get_version", &LBHdrV2::get_version)
        .def("get_nextProto", &LBHdrV2::get_nextProto)
        .def("get_entropy", &LBHdrV2::get_entropy)
        .def("get_eventNum", &LBHdrV2::get_eventNum)
        .def("get_fields", &LBHdrV2::get_Fields)
        .def("to_bytes", [](const LBHdrV2 &h) { return py::bytes(reinterpret_cast<const char *>(&h), sizeof(h)); });
    py::class_<LBHdrV3>(m, "LBHdrV3")
        .def(py::init<>())
        .def("set", &LBHdrV3::set, py::arg("slot_select") = 0, py::arg("port_select") = 0, py::arg("tick") = 0)
        .def("get_version", &LBHdrV3::get_version)
        .def("get_nextProto", &LBHdrV3::get_nextProto)
        .def("get_slotSelect", &LBHdrV3::get_slotSelect)
        .def("get_portSelect", &LBHdrV3::get_portSelect)
        .def("get_tick", &LBHdrV3::get_tick)
        .def("get_fields", &LBHdrV3::get_Fields)
        .def("to_bytes", [](const LBHdrV3 &h) { return py::bytes(reinterpret_cast<const char *>(&h), sizeof(h)); });
    py::class_<LBREHdr>(m, "LBREHdr").def(py::init<>());
    py::class_<SyncHdr>(m, "SyncHdr")
        .def(py::init<>())
        .def("set", &SyncHdr::set, py::arg("event_src_id") = 0, py::arg("event_num") = 0,
             py::arg("avg_rate") = 0, py::arg("unix_time_nano") = 0)
        .def("get_eventSrcId", &SyncHdr::get_eventSrcId)
        .def("get_eventNumber", &SyncHdr::get_eventNumber)
        .def("get_avgEventRateHz", &SyncHdr::get_avgEventRateHz)
        .def("get_unixTimeNano", &SyncHdr::get_unixTimeNano)
        .def("get_fields", &SyncHdr::get_Fields)
        .def("to_bytes", [](const SyncHdr &h) { return py::bytes(reinterpret_cast<const char *>(&h), sizeof(h)); });

    // ---- DataPlane (py_e2sarDP.cpp) ----
    py::module_ dp = m.def_submodule("DataPlane", "E2SAR DataPlane submodule (gfx950 SAR path)");

    py::class_<Segmenter> seg(dp, "Segmenter");
    py::class_<SegmenterFlagsT>(seg, "SegmenterFlags")
        .def(py::init<>())
        .def_readwrite("dpV6", &SegmenterFlagsT::dpV6)
        .def_readwrite("connectedSocket", &SegmenterFlagsT::connectedSocket)
        .def_readwrite("useCP", &SegmenterFlagsT::useCP)
        .def_readwrite("warmUpMs", &SegmenterFlagsT::warmUpMs)
        .def_readwrite("syncPeriodMs", &SegmenterFlagsT::syncPeriodMs)
        .def_readwrite("syncPeriods", &SegmenterFlagsT::syncPeriods)
        .def_readwrite("mtu", &SegmenterFlagsT::mtu)
        .def_readwrite("numSendSockets", &SegmenterFlagsT::numSendSockets)
        .def_readwrite("sndSocketBufSize", &SegmenterFlagsT::sndSocketBufSize)
        .def_readwrite("rateGbps", &SegmenterFlagsT::rateGbps)
        .def_readwrite("smooth", &SegmenterFlagsT::smooth)
        .def_readwrite("multiPort", &SegmenterFlagsT::multiPort)
        .def_readwrite("ticksAsREEventNum", &SegmenterFlagsT::ticksAsREEventNum)
        .def_readwrite("lbHdrVersion", &SegmenterFlagsT::lbHdrVersion)
        .def_readwrite("gpuDevice", &SegmenterFlagsT::gpuDevice)
        .def_readwrite("maxBatchEvents", &SegmenterFlagsT::maxBatchEvents)
        .def_static("getFromINI", &SegmenterFlagsT::getFromINI);
    seg.def(py::init<const EjfatURI &, uint16_t, uint32_t, const SegmenterFlagsT &>(), py::arg("uri"),
            py::arg("data_id"), py::arg("eventSrc_id"), py::arg("sflags") = SegmenterFlagsT());
    seg.def(py::init<const EjfatURI &, uint16_t, uint32_t, std::vector<int>, const SegmenterFlagsT &>(),
            py::arg("uri"), py::arg("data_id"), py::arg("eventSrc_id"), py::arg("cpu_core_list"),
            py::arg("sflags") = SegmenterFlagsT());
    seg.def("OpenAndStart", &Segmenter::openAndStart);
    seg.def(
        "sendEvent",
        [](Segmenter &s, py::buffer b, size_t len, EventNum_t ev, uint16_t did, uint16_t ent) {
            py::buffer_info bi = b.request();
            py::gil_scoped_release rel;
            return s.sendEvent(static_cast<uint8_t *>(bi.ptr), len, ev, did, ent);
        },
        py::arg("send_buf"), py::arg("buf_len"), py::arg("_eventNum") = 0LL, py::arg("_dataId") = 0,
        py::arg("entropy") = 0);
    seg.def(
        "sendNumpyArray",
        [](Segmenter &s, py::array a, size_t nbytes, EventNum_t ev, uint16_t did, uint16_t ent) {
            py::buffer_info bi = a.request();
            py::gil_scoped_release rel;
            return s.sendEvent(static_cast<uint8_t *>(bi.ptr), nbytes, ev, did, ent);
        },
        py::arg("numpy_array"), py::arg("nbytes"), py::arg("event_num") = 0LL, py::arg("data_id") = 0,
        py::arg("entropy") = 0);
    auto queue = [](Segmenter &s, py::buffer b, size_t bytes, int64_t ev, uint16_t did, uint16_t ent,
                    py::object cb, py::object arg) {
        py::buffer_info bi = b.request();
        void (*ccb)(std::any) = nullptr;
        std::any carg;
        if (!cb.is_none()) {
            ccb = PyCallback::execute;
            carg = new PyCallback{cb, arg};
        }
        auto res = s.addToSendQueue(static_cast<uint8_t *>(bi.ptr), bytes, (EventNum_t)ev, did, ent, ccb, carg);
        if (res.has_error() && ccb) delete std::any_cast<PyCallback *>(carg);   // refused: never called back
        return res;
    };
    seg.def("addNumpyArrayToSendQueue", queue, py::arg("numpy_array"), py::arg("nbytes"), py::arg("_eventNum") = 0LL,
            py::arg("_dataId") = 0, py::arg("entropy") = 0, py::arg("callback") = py::none(),
            py::arg("cbArg") = py::none());
    seg.def("addToSendQueue", queue, py::arg("send_buf"), py::arg("buf_len"), py::arg("_eventNum") = 0LL,
            py::arg("_dataId") = 0, py::arg("entropy") = 0, py::arg("callback") = py::none(),
            py::arg("cbArg") = py::none());
    py::class_<Segmenter::ReportedStats>(seg, "ReportedStats")
        .def_readonly("msgCnt", &Segmenter::ReportedStats::msgCnt)
        .def_readonly("errCnt", &Segmenter::ReportedStats::errCnt)
        .def_readonly("lastErrno", &Segmenter::ReportedStats::lastErrno)
        .def_readonly("lastE2SARError", &Segmenter::ReportedStats::lastE2SARError);
    seg.def("getSendStats", &Segmenter::getSendStats);
    seg.def("getSyncStats", &Segmenter::getSyncStats);
    seg.def("getMTU", &Segmenter::getMTU);
    seg.def("getMaxPldLen", &Segmenter::getMaxPldLen);
    seg.def("getIntf", &Segmenter::getIntf);
    seg.def("stopThreads", [](Segmenter &s) {
        py::gil_scoped_release rel;
        s.stopThreads();
    });

    py::class_<Reassembler> reas(dp, "Reassembler");
    py::class_<ReassemblerFlagsT>(reas, "ReassemblerFlags")
        .def(py::init<>())
        .def_readwrite("useCP", &ReassemblerFlagsT::useCP)
        .def_readwrite("useHostAddress", &ReassemblerFlagsT::useHostAddress)
        .def_readwrite("period_ms", &ReassemblerFlagsT::period_ms)
        .def_readwrite("validateCert", &ReassemblerFlagsT::validateCert)
        .def_readwrite("Ki", &ReassemblerFlagsT::Ki)
        .def_readwrite("Kp", &ReassemblerFlagsT::Kp)
        .def_readwrite("Kd", &ReassemblerFlagsT::Kd)
        .def_readwrite("setPoint", &ReassemblerFlagsT::setPoint)
        .def_readwrite("epoch_ms", &ReassemblerFlagsT::epoch_ms)
        .def_readwrite("portRange", &ReassemblerFlagsT::portRange)
        .def_readwrite("withLBHeader", &ReassemblerFlagsT::withLBHeader)
        .def_readwrite("eventTimeout_ms", &ReassemblerFlagsT::eventTimeout_ms)
        .def_readwrite("rcvSocketBufSize", &ReassemblerFlagsT::rcvSocketBufSize)
        .def_readwrite("weight", &ReassemblerFlagsT::weight)
        .def_readwrite("min_factor", &ReassemblerFlagsT::min_factor)
        .def_readwrite("max_factor", &ReassemblerFlagsT::max_factor)
        .def_readwrite("gpuDevice", &ReassemblerFlagsT::gpuDevice)
        .def_readwrite("recvBatch", &ReassemblerFlagsT::recvBatch)
        .def_readwrite("referenceOrder", &ReassemblerFlagsT::referenceOrder)
        .def_readwrite("recvStride", &ReassemblerFlagsT::recvStride)
        .def_readwrite("tableSlots", &ReassemblerFlagsT::tableSlots)
        .def_readwrite("arenaBytes", &ReassemblerFlagsT::arenaBytes)
        .def_readwrite("batchTimeout_us", &ReassemblerFlagsT::batchTimeout_us)
        .def_static("getFromINI", &ReassemblerFlagsT::getFromINI);
    reas.def(py::init([](const EjfatURI &u, const IPAddress &ip, uint16_t port, size_t n, const ReassemblerFlagsT &f) {
                 return new Reassembler(u, ip.s, port, n, f);
             }),
             py::arg("uri"), py::arg("data_ip"), py::arg("starting_port"), py::arg("num_recv_threads") = (size_t)1,
             py::arg("rflags") = ReassemblerFlagsT());
    reas.def(py::init<const EjfatURI &, uint16_t, size_t, const ReassemblerFlagsT &, bool>(), py::arg("uri"),
             py::arg("starting_port"), py::arg("num_recv_threads") = (size_t)1, py::arg("rflags") = ReassemblerFlagsT(),
             py::arg("v6") = false);
    reas.def(py::init([](const EjfatURI &u, const IPAddress &ip, uint16_t port, std::vector<int> cores,
                         const ReassemblerFlagsT &f) { return new Reassembler(u, ip.s, port, cores, f); }),
             py::arg("uri"), py::arg("data_ip"), py::arg("starting_port"), py::arg("cpu_core_list"),
             py::arg("rflags") = ReassemblerFlagsT());
    reas.def(py::init<const EjfatURI &, uint16_t, std::vector<int>, const ReassemblerFlagsT &, bool>(), py::arg("uri"),
             py::arg("starting_port"), py::arg("cpu_core_list"), py::arg("rflags") = ReassemblerFlagsT(),
             py::arg("v6") = false);
    reas.def("getEventBytes", [](Reassembler &r) {
        uint8_t *b = nullptr;
        size_t n = 0;
        EventNum_t ev = 0;
        uint16_t d = 0;
        auto res = r.getEvent(&b, &n, &ev, &d);
        return event_tuple_bytes(res, b, n, ev, d);
    });
    reas.def(
        "recvEventBytes",
        [](Reassembler &r, uint64_t wait_ms) {
            uint8_t *b = nullptr;
            size_t n = 0;
            EventNum_t ev = 0;
            uint16_t d = 0;
            result<int> res = 0;
            {
                py::gil_scoped_release rel;
                res = r.recvEvent(&b, &n, &ev, &d, wait_ms);
            }
            return event_tuple_bytes(res, b, n, ev, d);
        },
        py::arg("wait_ms") = 0);
    reas.def(
        "get1DNumpyArray",
        [](Reassembler &r, py::dtype dt) {
            uint8_t *b = nullptr;
            size_t n = 0;
            EventNum_t ev = 0;
            uint16_t d = 0;
            auto res = r.getEvent(&b, &n, &ev, &d);
            return event_tuple_array(res, b, n, ev, d, dt);
        },
        py::arg("data_type"));
    reas.def(
        "recv1DNumpyArray",
        [](Reassembler &r, py::dtype dt, uint64_t wait_ms) {
            uint8_t *b = nullptr;
            size_t n = 0;
            EventNum_t ev = 0;
            uint16_t d = 0;
            result<int> res = 0;
            {
                py::gil_scoped_release rel;
                res = r.recvEvent(&b, &n, &ev, &d, wait_ms);
            }
            return event_tuple_array(res, b, n, ev, d, dt);
        },
        py::arg("data_type"), py::arg("wait_ms") = 0);
    reas.def("OpenAndStart", &Reassembler::openAndStart);
    reas.def("registerWorker", &Reassembler::registerWorker);
    reas.def("deregisterWorker", &Reassembler::deregisterWorker);
    reas.def("get_FDStats", &Reassembler::get_FDStats);
    reas.def("get_LostEvent", [](Reassembler &r) -> py::tuple {
        auto res = r.get_LostEvent();
        if (res.has_error()) return py::make_tuple();
        auto t = res.value();
        return py::make_tuple(std::get<0>(t), std::get<1>(t), std::get<2>(t));
    });
    py::class_<Reassembler::ReportedStats>(reas, "ReportedStats")
        .def_readonly("enqueueLoss", &Reassembler::ReportedStats::enqueueLoss)
        .def_readonly("reassemblyLoss", &Reassembler::ReportedStats::reassemblyLoss)
        .def_readonly("eventSuccess", &Reassembler::ReportedStats::eventSuccess)
        .def_readonly("lastErrno", &Reassembler::ReportedStats::lastErrno)
        .def_readonly("grpcErrCnt", &Reassembler::ReportedStats::grpcErrCnt)
        .def_readonly("dataErrCnt", &Reassembler::ReportedStats::dataErrCnt)
        .def_readonly("lastE2SARError", &Reassembler::ReportedStats::lastE2SARError)
        .def_readonly("totalPackets", &Reassembler::ReportedStats::totalPackets)
        .def_readonly("totalBytes", &Reassembler::ReportedStats::totalBytes)
        .def_readonly("badHeaderDiscards", &Reassembler::ReportedStats::badHeaderDiscards);
    reas.def("getStats", &Reassembler::getStats);
    reas.def("get_dataIP", &Reassembler::get_dataIP);
    py::class_<Reassembler::DeviceStats>(reas, "DeviceStats")
        .def_readonly("tableUsed", &Reassembler::DeviceStats::tableUsed)
        .def_readonly("arenaUsed", &Reassembler::DeviceStats::arenaUsed)
        .def_readonly("upkeeps", &Reassembler::DeviceStats::upkeeps)
        .def_readonly("inProgress", &Reassembler::DeviceStats::inProgress)
        .def_readonly("errorFlags", &Reassembler::DeviceStats::errorFlags);
    reas.def("getDeviceStats", &Reassembler::getDeviceStats);
    reas.def("get_numRecvThreads", &Reassembler::get_numRecvThreads);
    reas.def("get_recvPorts", &Reassembler::get_recvPorts);
    reas.def("get_portRange", &Reassembler::get_portRange);
    reas.def("stopThreads", [](Reassembler &r) {
        py::gil_scoped_release rel;
        r.stopThreads();
    });
}
