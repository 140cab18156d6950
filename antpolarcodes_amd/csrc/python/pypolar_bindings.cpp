// pypolar_bindings.cpp -- pybind11 module `_pypolar` with the reference's `pypolar`
// surface (python/bindings/*.cc of david13pod/antPolarCodes): PolarDecoder,
// PolarEncoder, Detector, Puncturer, frozen_bits -- same names, arguments and error messages --
// plus PolarDecoder.decode_batch / decode_device for batched GPU decoding.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <type_traits>
#include <pybind11/stl.h>

#include <polarcode/construction/constructor.h>
#include <polarcode/decoding/decoder.h>
#include <polarcode/encoding/butterfly_fip_packed.h>
#include <polarcode/encoding/encoder.h>
#include <polarcode/errordetection/errordetector.h>
#include <polarcode/puncturer.h>

#include <cstring>
#include <memory>

namespace py = pybind11;
using namespace PolarCode;

namespace {

// The decoder does not own its detector (as in the reference); the Python wrapper
// keeps the detector alive instead of leaking one per setErrorDetection call.
struct PyDecoder {
    std::unique_ptr<Decoding::Decoder> dec;
    std::unique_ptr<ErrorDetection::Detector> det;
};

struct PyEncoder {
    std::unique_ptr<Encoding::ButterflyFipPacked> enc;
    std::unique_ptr<ErrorDetection::Detector> det;
};

using f32array = py::array_t<float, py::array::c_style | py::array::forcecast>;
using u8array = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;
using f64array = py::array_t<double, py::array::c_style | py::array::forcecast>;
using i8array = py::array_t<int8_t, py::array::c_style | py::array::forcecast>;

// decode_batch over float32 or int8 frames (F x N): info [, ok] [, metrics]
template <typename T>
py::object decode_batch_impl(PyDecoder& s, const py::array_t<T, py::array::c_style | py::array::forcecast>& a,
                             bool return_ok, bool return_metrics)
{
    py::buffer_info in = a.request();
    const size_t N = s.dec->blockLength(), L = s.dec->getListSize();
    if (in.ndim != 2 || (size_t)in.shape[1] != N)
        throw std::runtime_error("decode_batch expects a (frames, blockLength) float32 or int8 array");
    const size_t F = (size_t)in.shape[0], kb = (s.dec->infoLength() + 7) / 8;
    py::array_t<uint8_t> info({ F, kb });
    py::array_t<uint8_t> ok(F);
    py::array_t<float> met({ F, L });
    {
        py::gil_scoped_release nogil;
        if constexpr (std::is_same<T, float>::value)
            s.dec->decodeBatch(static_cast<const float*>(in.ptr), F, info.mutable_data(), ok.mutable_data(),
                               return_metrics ? met.mutable_data() : nullptr);
        else
            s.dec->decodeBatchI8(static_cast<const int8_t*>(in.ptr), F, info.mutable_data(), ok.mutable_data(),
                                 return_metrics ? met.mutable_data() : nullptr);
    }
    if (!return_ok && !return_metrics)
        return std::move(info);
    py::tuple t(1 + (return_ok ? 1 : 0) + (return_metrics ? 1 : 0));
    size_t k = 0;
    t[k++] = info;
    if (return_ok)
        t[k++] = ok;
    if (return_metrics)
        t[k++] = met;
    return std::move(t);
}

// Puncturer.puncture / depuncture for one element type (puncturer_python.cc:37-160)
template <typename T>
py::array_t<T> do_puncture(Puncturer& self, const py::array_t<T, py::array::c_style | py::array::forcecast>& a)
{
    py::buffer_info in = a.request();
    if (in.ndim != 1)
        throw std::runtime_error("Only ONE-dimensional vectors allowed!");
    if ((size_t)in.size != self.parentBlockLength())
        throw std::runtime_error("Input vector size != parentBlockSize!");
    auto res = py::array_t<T>(self.blockLength());
    self.puncture<T>(res.mutable_data(), static_cast<const T*>(in.ptr));
    return res;
}

template <typename T>
py::array_t<T> do_depuncture(Puncturer& self,
                             const py::array_t<T, py::array::c_style | py::array::forcecast>& a,
                             const char* sizeMsg)
{
    py::buffer_info in = a.request();
    if (in.ndim != 1)
        throw std::runtime_error("Only ONE-dimensional vectors allowed!");
    if ((size_t)in.size != self.blockLength())
        throw std::runtime_error(sizeMsg);
    auto res = py::array_t<T>(self.parentBlockLength());
    self.depuncture<T>(res.mutable_data(), static_cast<const T*>(in.ptr));
    return res;
}

} // namespace

PYBIND11_MODULE(_pypolar, m)
{
    m.doc() = "MI355X polar SC/SCL decoding with the reference pypolar API";

    py::class_<PyDecoder>(m, "PolarDecoder")
        .def(py::init([](size_t N, size_t L, std::vector<unsigned> frozen, std::string type) {
                 auto d = std::make_unique<PyDecoder>();
                 d->dec.reset(Decoding::create(N, L, frozen, type));
                 // makeDecoder installs a CRC-8 the decoder does not own; adopt it here
                 d->det = std::make_unique<ErrorDetection::CRC8>();
                 d->dec->setErrorDetection(d->det.get());
                 return d;
             }),
             py::arg("blockLength"), py::arg("listSize"), py::arg("frozenBitPositions"), py::arg("decoderType"))
        .def("blockLength", [](PyDecoder& s) { return s.dec->blockLength(); })
        .def("infoLength", [](PyDecoder& s) { return s.dec->infoLength(); })
        .def("listSize", [](PyDecoder& s) { return s.dec->getListSize(); })
        .def("setSystematic", [](PyDecoder& s, bool v) { s.dec->setSystematic(v); })
        .def("isSystematic", [](PyDecoder& s) { return s.dec->isSystematic(); })
        .def("frozenBits", [](PyDecoder& s) { return s.dec->frozenBits(); })
        .def("getErrorDetectionMode", [](PyDecoder& s) { return s.dec->getErrorDetectionMode(); })
        .def(
            "setErrorDetection",
            [](PyDecoder& s, unsigned size, std::string type) {
                std::unique_ptr<ErrorDetection::Detector> d(ErrorDetection::create(size, type));
                s.dec->setErrorDetection(d.get());
                s.det = std::move(d);
            },
            py::arg("size") = 0, py::arg("type") = "crc")
        .def("decode_vector",
             [](PyDecoder& s, const f32array& a) {
                 py::buffer_info in = a.request();
                 if (in.ndim != 1)
                     throw std::runtime_error("Only ONE-dimensional vectors allowed!");
                 if ((size_t)in.size != s.dec->blockLength())
                     throw std::runtime_error("Input vector size != blockSize // 8!");
                 auto res = py::array_t<uint8_t>(s.dec->infoLength() / 8);
                 std::vector<uint8_t> tmp(s.dec->infoLength() / 8 + 8);
                 s.dec->decode_vector(static_cast<const float*>(in.ptr), tmp.data());
                 std::memcpy(res.request().ptr, tmp.data(), s.dec->infoLength() / 8);
                 return res;
             })
        .def("decode_vector", // the reference's int8 overload (decoder_python.cc:58-74)
             [](PyDecoder& s, const i8array& a) {
                 py::buffer_info in = a.request();
                 if (in.ndim != 1)
                     throw std::runtime_error("Only ONE-dimensional vectors allowed!");
                 if ((size_t)in.size != s.dec->blockLength())
                     throw std::runtime_error("Input vector size != blockSize // 8!");
                 auto res = py::array_t<uint8_t>(s.dec->infoLength() / 8);
                 std::vector<uint8_t> tmp(s.dec->infoLength() / 8 + 8);
                 s.dec->decode_vector(static_cast<const char*>(in.ptr), tmp.data());
                 std::memcpy(res.request().ptr, tmp.data(), s.dec->infoLength() / 8);
                 return res;
             })
        .def("getSoftCodeword", // Decoder::getSoftCodeword after decode_vector: float32 (float
                                // decoders) or int8 (8-bit decoders) per codeword bit
             [](PyDecoder& s) -> py::object {
                 if (dynamic_cast<CharContainer*>(s.dec->outputContainer())) {
                     py::array_t<int8_t> out(s.dec->blockLength());
                     s.dec->getSoftCodeword(out.mutable_data());
                     return std::move(out);
                 }
                 py::array_t<float> out(s.dec->blockLength());
                 s.dec->getSoftCodeword(out.mutable_data());
                 return std::move(out);
             })
        .def("getSoftInformation",
             [](PyDecoder& s) -> py::object {
                 if (dynamic_cast<CharContainer*>(s.dec->outputContainer())) {
                     py::array_t<int8_t> out(s.dec->infoLength());
                     s.dec->getSoftInformation(out.mutable_data());
                     return std::move(out);
                 }
                 py::array_t<float> out(s.dec->infoLength());
                 s.dec->getSoftInformation(out.mutable_data());
                 return std::move(out);
             })
        .def("carriedMetric", // SCL: path 0's metric the next decode_vector starts from (Q8)
             [](PyDecoder& s) {
                 auto* g = dynamic_cast<Decoding::GpuDecoder*>(s.dec.get());
                 return g ? g->carriedMetric() : 0.0f;
             })
        .def(
            "decode_batch",
            [](PyDecoder& s, const f32array& a, bool return_ok, bool return_metrics) {
                return decode_batch_impl<float>(s, a, return_ok, return_metrics);
            },
            py::arg("llrs"), py::arg("return_ok") = false, py::arg("return_metrics") = false)
        .def(
            "decode_batch",
            [](PyDecoder& s, const i8array& a, bool return_ok, bool return_metrics) {
                return decode_batch_impl<int8_t>(s, a, return_ok, return_metrics);
            },
            py::arg("llrs"), py::arg("return_ok") = false, py::arg("return_metrics") = false)
        .def("isFixedPoint",
             [](PyDecoder& s) {
                 auto* g = dynamic_cast<Decoding::GpuDecoder*>(s.dec.get());
                 return g != nullptr && g->isFixedPoint();
             })
        .def(
            "decode_device_i8",
            [](PyDecoder& s, uintptr_t llr, size_t F, uintptr_t info, uintptr_t ok, uintptr_t metrics,
               uintptr_t stream) {
                auto* g = dynamic_cast<Decoding::GpuDecoder*>(s.dec.get());
                if (!g)
                    throw std::logic_error("not a GPU decoder");
                g->decodeBatchDeviceI8(reinterpret_cast<const int8_t*>(llr), F, reinterpret_cast<uint8_t*>(info),
                                       reinterpret_cast<uint8_t*>(ok), reinterpret_cast<float*>(metrics),
                                       reinterpret_cast<void*>(stream));
            },
            py::arg("llr_ptr"), py::arg("frames"), py::arg("info_ptr"), py::arg("ok_ptr") = 0,
            py::arg("metrics_ptr") = 0, py::arg("stream") = 0)
        .def(
            "decode_device",
            [](PyDecoder& s, uintptr_t llr, size_t F, uintptr_t info, uintptr_t ok, uintptr_t metrics,
               uintptr_t stream) {
                s.dec->decodeBatchDevice(reinterpret_cast<const float*>(llr), F, reinterpret_cast<uint8_t*>(info),
                                         reinterpret_cast<uint8_t*>(ok), reinterpret_cast<float*>(metrics),
                                         reinterpret_cast<void*>(stream));
            },
            py::arg("llr_ptr"), py::arg("frames"), py::arg("info_ptr"), py::arg("ok_ptr") = 0,
            py::arg("metrics_ptr") = 0, py::arg("stream") = 0);

    py::class_<PyEncoder>(m, "PolarEncoder")
        .def(py::init([](size_t N, std::vector<unsigned> frozen) {
                 auto e = std::make_unique<PyEncoder>();
                 e->enc = std::make_unique<Encoding::ButterflyFipPacked>(N, frozen);
                 return e;
             }),
             py::arg("blockLength"), py::arg("frozenBitPositions"))
        .def("blockLength", [](PyEncoder& s) { return s.enc->blockLength(); })
        .def("infoLength", [](PyEncoder& s) { return s.enc->infoLength(); })
        .def("setSystematic", [](PyEncoder& s, bool v) { s.enc->setSystematic(v); })
        .def("isSystematic", [](PyEncoder& s) { return s.enc->isSystematic(); })
        .def("frozenBits", [](PyEncoder& s) { return s.enc->frozenBits(); })
        .def("getErrorDetectionMode", [](PyEncoder& s) { return s.enc->getErrorDetectionMode(); })
        .def(
            "setErrorDetection",
            [](PyEncoder& s, unsigned size, std::string type) {
                std::unique_ptr<ErrorDetection::Detector> d(ErrorDetection::create(size, type));
                s.enc->setErrorDetection(d.get());
                s.det = std::move(d);
            },
            py::arg("size") = 0, py::arg("type") = "crc")
        .def("encode_vector", [](PyEncoder& s, const u8array& a) {
            py::buffer_info in = a.request();
            if (in.ndim != 1)
                throw std::runtime_error("Only ONE-dimensional vectors allowed!");
            if ((size_t)in.size != s.enc->infoLength() / 8)
                throw std::runtime_error("Input vector size != infoSize // 8!");
            std::vector<uint8_t> info(static_cast<uint8_t*>(in.ptr), static_cast<uint8_t*>(in.ptr) + in.size);
            info.resize(info.size() + 8);
            auto res = py::array_t<uint8_t>(s.enc->blockLength() / 8);
            s.enc->encode_vector(info.data(), res.mutable_data());
            return res;
        });

    py::class_<ErrorDetection::Detector>(m, "Detector")
        .def(py::init(&ErrorDetection::create), py::arg("size"), py::arg("type"))
        .def("getCheckBitCount", &ErrorDetection::Detector::getCheckBitCount)
        .def("generate",
             [](ErrorDetection::Detector& self, const u8array& a) {
                 py::buffer_info in = a.request();
                 if (in.ndim != 1)
                     throw std::runtime_error("Only ONE-dimensional vectors allowed!");
                 // byte-sized checksums are appended (detector_python.cc); CRC-11 (this
                 // build's extension) writes its 11 bits over the tail of the given bytes
                 const unsigned cb = self.getCheckBitCount();
                 auto res = py::array_t<uint8_t>(in.size + (cb % 8 ? 0 : cb / 8));
                 py::buffer_info rb = res.request();
                 std::memcpy(rb.ptr, in.ptr, in.size);
                 self.generate(rb.ptr, (int)rb.size);
                 return res;
             })
        .def("check", [](ErrorDetection::Detector& self, const u8array& a) {
            py::buffer_info in = a.request();
            if (in.ndim != 1)
                throw std::runtime_error("Only ONE-dimensional vectors allowed!");
            std::vector<uint8_t> tmp(static_cast<uint8_t*>(in.ptr), static_cast<uint8_t*>(in.ptr) + in.size);
            return self.check(tmp.data(), (int)tmp.size());
        });

    // overload order as the reference registers them: double, float, uint8
    py::class_<Puncturer>(m, "Puncturer")
        .def(py::init<size_t, std::vector<unsigned>>(), py::arg("blockLength"), py::arg("frozenBitPositions"))
        .def("blockLength", &Puncturer::blockLength)
        .def("parentBlockLength", &Puncturer::parentBlockLength)
        .def("blockOutputPositions", &Puncturer::blockOutputPositions)
        .def("puncturePacked",
             [](Puncturer& self, const u8array& a) {
                 py::buffer_info in = a.request();
                 if (in.ndim != 1)
                     throw std::runtime_error("Only ONE-dimensional vectors allowed!");
                 if ((size_t)in.size != self.parentBlockLength() / 8)
                     throw std::runtime_error("Input vector size != parentBlockSize!");
                 auto res = py::array_t<uint8_t>(self.blockLength() / 8);
                 self.puncturePacked(res.mutable_data(), static_cast<const uint8_t*>(in.ptr));
                 return res;
             })
        .def("puncture", [](Puncturer& s, const f64array& a) { return do_puncture<double>(s, a); })
        .def("puncture", [](Puncturer& s, const f32array& a) { return do_puncture<float>(s, a); })
        .def("puncture", [](Puncturer& s, const u8array& a) { return do_puncture<uint8_t>(s, a); })
        .def("depuncture",
             [](Puncturer& s, const f64array& a) { return do_depuncture<double>(s, a, "Input vector size != blockSize!"); })
        .def("depuncture",
             [](Puncturer& s, const f32array& a) { return do_depuncture<float>(s, a, "Input vector size != blockSize!"); })
        .def("depuncture", [](Puncturer& s, const u8array& a) {
            return do_depuncture<uint8_t>(s, a, "Input vector size != bBlockSize!");
        });

    m.def("frozen_bits", &Construction::frozen_bits, py::arg("blockLength"), py::arg("infoLength"),
          py::arg("designSNR"), py::arg("constructorType") = std::string("BB"));
}
