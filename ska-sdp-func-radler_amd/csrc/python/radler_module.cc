// The `radler` Python module of the MI355X build: the reference's pybind11
// surface (python/pywrappers.cc, pysettings.cc, pywork_table.cc,
// pyradler.cc, pycomponent_list.cc) over libradler_amd, plus `radler.gpu`
// helpers for device-resident runs (bench / tests).
#include <pybind11/iostream.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <sstream>

#include "communicator.h"
#include "device.h"
#include "device_run.h"
#include "dijkstra_splitter.h"
#include "image_accessors.h"
#include "logger.h"
#include "radler.h"
#include "rms_image.h"
#include "component_optimization.h"
#include "fft_sizes.h"
#include "host_profile.h"
#include "multiscale_transforms.h"
#include "subminor.h"

namespace py = pybind11;
using AccessorList = std::vector<std::unique_ptr<aocommon::ImageAccessor>>;
PYBIND11_MAKE_OPAQUE(AccessorList)

namespace {

using FloatArray = py::array_t<float, py::array::c_style>;

template <class T>
std::unique_ptr<T> MakeAccessor(FloatArray& data) {
  if (data.ndim() != 2)
    throw std::runtime_error("Provided array should have 2 dimensions.");
  aocommon::Image view(data.mutable_data(), size_t(data.shape(1)),
                       size_t(data.shape(0)));
  return std::make_unique<T>(view);
}

void InitSettings(py::module& m) {  // python/pysettings.cc
  py::enum_<radler::AlgorithmType>(m, "AlgorithmType")
      .value("generic_clean", radler::AlgorithmType::kGenericClean)
      .value("multiscale", radler::AlgorithmType::kMultiscale)
      .value("iuwt", radler::AlgorithmType::kIuwt)
      .value("more_sane", radler::AlgorithmType::kMoreSane)
      .value("python", radler::AlgorithmType::kPython);
  py::enum_<radler::OptimizationAlgorithm>(m, "OptimizationAlgorithm")
      .value("clean", radler::OptimizationAlgorithm::kClean)
      .value("linear_equation_solver", radler::OptimizationAlgorithm::kLinearEquationSolver)
      .value("gradient_descent", radler::OptimizationAlgorithm::kGradientDescent)
      .value("regularized_gradient_descent",
             radler::OptimizationAlgorithm::kRegularizedGradientDescent);
  py::enum_<radler::LocalRmsMethod>(m, "LocalRmsMethod")
      .value("none", radler::LocalRmsMethod::kNone)
      .value("rms_window", radler::LocalRmsMethod::kRmsWindow)
      .value("rms_and_minimum_window", radler::LocalRmsMethod::kRmsAndMinimumWindow);
  py::enum_<radler::MultiscaleShape>(m, "MultiscaleShape")
      .value("tapered_quadratic", radler::MultiscaleShape::kTaperedQuadraticShape)
      .value("gaussian", radler::MultiscaleShape::kGaussianShape);

  py::class_<radler::Settings> settings(m, "Settings");
  settings.def(py::init<>())
      .def_readwrite("trimmed_image_width", &radler::Settings::trimmed_image_width)
      .def_readwrite("trimmed_image_height", &radler::Settings::trimmed_image_height)
      .def_readwrite("channels_out", &radler::Settings::channels_out)
      .def_readwrite("pixel_scale", &radler::Settings::pixel_scale)
      .def_readwrite("thread_count", &radler::Settings::thread_count)
      .def_readwrite("prefix_name", &radler::Settings::prefix_name)
      .def_readwrite("linked_polarizations", &radler::Settings::linked_polarizations)
      .def_readwrite("parallel", &radler::Settings::parallel)
      .def_readwrite("absolute_threshold", &radler::Settings::absolute_threshold)
      .def_readwrite("minor_loop_gain", &radler::Settings::minor_loop_gain)
      .def_readwrite("major_loop_gain", &radler::Settings::major_loop_gain)
      .def_readwrite("auto_threshold_sigma", &radler::Settings::auto_threshold_sigma)
      .def_readwrite("auto_mask_sigma", &radler::Settings::auto_mask_sigma)
      .def_readwrite("absolute_auto_mask_threshold",
                     &radler::Settings::absolute_auto_mask_threshold)
      .def_readwrite("save_source_list", &radler::Settings::save_source_list)
      .def_readwrite("minor_iteration_count", &radler::Settings::minor_iteration_count)
      .def_readwrite("major_iteration_count", &radler::Settings::major_iteration_count)
      .def_readwrite("divergence_limit", &radler::Settings::divergence_limit)
      .def_readwrite("allow_negative_components",
                     &radler::Settings::allow_negative_components)
      .def_readwrite("stop_on_negative_components",
                     &radler::Settings::stop_on_negative_components)
      .def_readwrite("squared_joins", &radler::Settings::squared_joins)
      .def_readwrite("spectral_correction_frequency",
                     &radler::Settings::spectral_correction_frequency)
      .def_readwrite("spectral_correction", &radler::Settings::spectral_correction)
      .def_readwrite("border_ratio", &radler::Settings::border_ratio)
      .def_readwrite("fits_mask", &radler::Settings::fits_mask)
      .def_readwrite("casa_mask", &radler::Settings::casa_mask)
      .def_readwrite("horizon_mask_distance", &radler::Settings::horizon_mask_distance)
      .def_readwrite("horizon_mask_filename", &radler::Settings::horizon_mask_filename)
      .def_readwrite("local_rms", &radler::Settings::local_rms)
      .def_readwrite("spectral_fitting", &radler::Settings::spectral_fitting)
      .def_readwrite("algorithm_type", &radler::Settings::algorithm_type)
      .def_readwrite("generic", &radler::Settings::generic)
      .def_readwrite("multiscale", &radler::Settings::multiscale)
      .def_readwrite("more_sane", &radler::Settings::more_sane)
      .def_readwrite("python", &radler::Settings::python);

  py::class_<radler::Settings::Generic>(settings, "Generic")
      .def_readwrite("use_sub_minor_optimization",
                     &radler::Settings::Generic::use_sub_minor_optimization);
  py::class_<radler::Settings::Multiscale>(settings, "Multiscale")
      .def_readwrite("fast_sub_minor_loop", &radler::Settings::Multiscale::fast_sub_minor_loop)
      .def_readwrite("sub_minor_loop_gain", &radler::Settings::Multiscale::sub_minor_loop_gain)
      .def_readwrite("scale_bias", &radler::Settings::Multiscale::scale_bias)
      .def_readwrite("max_scales", &radler::Settings::Multiscale::max_scales)
      .def_readwrite("convolution_padding", &radler::Settings::Multiscale::convolution_padding)
      .def_readwrite("scale_list", &radler::Settings::Multiscale::scale_list)
      .def_readwrite("shape", &radler::Settings::Multiscale::shape);
  py::class_<radler::Settings::MoreSane>(settings, "MoreSane")
      .def_readwrite("location", &radler::Settings::MoreSane::location)
      .def_readwrite("arguments", &radler::Settings::MoreSane::arguments)
      .def_readwrite("sigma_levels", &radler::Settings::MoreSane::sigma_levels);
  py::class_<radler::Settings::Python>(settings, "Python")
      .def_readwrite("filename", &radler::Settings::Python::filename);
  py::class_<radler::Settings::Parallel>(settings, "Parallel")
      .def_readwrite("grid_width", &radler::Settings::Parallel::grid_width)
      .def_readwrite("grid_height", &radler::Settings::Parallel::grid_height)
      .def_readwrite("max_threads", &radler::Settings::Parallel::max_threads);
  py::class_<radler::Settings::PixelScale>(settings, "PixelScale")
      .def_readwrite("x", &radler::Settings::PixelScale::x)
      .def_readwrite("y", &radler::Settings::PixelScale::y);
  py::class_<radler::Settings::LocalRms>(settings, "LocalRms")
      .def_readwrite("method", &radler::Settings::LocalRms::method)
      .def_readwrite("window", &radler::Settings::LocalRms::window)
      .def_readwrite("image", &radler::Settings::LocalRms::image)
      .def_readwrite("strength", &radler::Settings::LocalRms::strength);
  py::class_<radler::Settings::SpectralFitting>(settings, "SpectralFitting")
      .def_readwrite("mode", &radler::Settings::SpectralFitting::mode)
      .def_readwrite("terms", &radler::Settings::SpectralFitting::terms)
      .def_readwrite("forced_filename", &radler::Settings::SpectralFitting::forced_filename);

  py::enum_<aocommon::PolarizationEnum>(m, "Polarization")
      .value("stokes_i", aocommon::PolarizationEnum::StokesI)
      .value("stokes_q", aocommon::PolarizationEnum::StokesQ)
      .value("stokes_u", aocommon::PolarizationEnum::StokesU)
      .value("stokes_v", aocommon::PolarizationEnum::StokesV)
      .value("rr", aocommon::PolarizationEnum::RR)
      .value("rl", aocommon::PolarizationEnum::RL)
      .value("lr", aocommon::PolarizationEnum::LR)
      .value("ll", aocommon::PolarizationEnum::LL)
      .value("xx", aocommon::PolarizationEnum::XX)
      .value("xy", aocommon::PolarizationEnum::XY)
      .value("yx", aocommon::PolarizationEnum::YX)
      .value("yy", aocommon::PolarizationEnum::YY)
      .value("full_stokes", aocommon::PolarizationEnum::FullStokes)
      .value("instrumental", aocommon::PolarizationEnum::Instrumental)
      .value("diagonal_instrumental", aocommon::PolarizationEnum::DiagonalInstrumental);
  py::enum_<schaapcommon::fitters::SpectralFittingMode>(m, "SpectralFittingMode")
      .value("no_fitting", schaapcommon::fitters::SpectralFittingMode::kNoFitting)
      .value("polynomial", schaapcommon::fitters::SpectralFittingMode::kPolynomial)
      .value("log_polynomial", schaapcommon::fitters::SpectralFittingMode::kLogPolynomial)
      .value("forced_terms", schaapcommon::fitters::SpectralFittingMode::kForcedTerms);
}

void InitSpectralFitter(py::module& m) {
  // schaapcommon::fitters::SpectralFitter (the reference binds fit /
  // fit_and_evaluate in python_deconvolution.cc:22-82, 153-155)
  using schaapcommon::fitters::SpectralFitter;
  using schaapcommon::fitters::SpectralFittingMode;
  py::class_<SpectralFitter>(m, "SpectralFitter")
      .def(py::init([](SpectralFittingMode mode, size_t n_terms,
                       const std::vector<double>& frequencies,
                       const std::vector<float>& weights) {
             return std::make_unique<SpectralFitter>(mode, n_terms, frequencies, weights);
           }),
           py::arg("mode"), py::arg("n_terms"), py::arg("frequencies"),
           py::arg("weights"))
      .def_property_readonly("mode", &SpectralFitter::Mode)
      .def_property_readonly("n_terms", &SpectralFitter::NTerms)
      .def_property_readonly("frequencies", &SpectralFitter::Frequencies)
      .def_property_readonly("weights", &SpectralFitter::Weights)
      .def_property_readonly("reference_frequency", &SpectralFitter::ReferenceFrequency)
      .def("fit",
           [](const SpectralFitter& self, const std::vector<float>& values, size_t x,
              size_t y) {
             if (values.size() != self.Frequencies().size())
               throw std::runtime_error("fit: one value per channel is required");
             std::vector<float> terms;
             self.Fit(terms, values.data(), x, y);
             return terms;
           },
           py::arg("values"), py::arg("x") = 0, py::arg("y") = 0)
      .def("fit_and_evaluate",
           [](const SpectralFitter& self, std::vector<float> values, size_t x, size_t y) {
             if (self.Mode() != SpectralFittingMode::kNoFitting &&
                 values.size() != self.Frequencies().size())
               throw std::runtime_error(
                   "fit_and_evaluate: one value per channel is required");
             std::vector<float> scratch;
             self.FitAndEvaluate(values.data(), x, y, scratch);
             return values;
           },
           py::arg("values"), py::arg("x") = 0, py::arg("y") = 0)
      .def("evaluate",
           [](const SpectralFitter& self, const std::vector<float>& terms,
              double frequency) { return self.Evaluate(terms, frequency); },
           py::arg("terms"), py::arg("frequency"));
}

void InitWorkTable(py::module& m) {  // python/pywork_table.cc
  py::class_<AccessorList>(m, "VectorUniquePtrImageAccessor")
      .def("__len__", [](const AccessorList& self) { return self.size(); })
      .def("append", [](AccessorList& self, FloatArray& psf) {
        self.emplace_back(MakeAccessor<radler::utils::LoadOnlyImageAccessor>(psf));
      });

  py::class_<radler::WorkTable>(m, "WorkTable")
      .def(py::init([](py::array_t<size_t> py_psf_offsets, size_t n_original_groups,
                       size_t n_deconvolution_groups, size_t channel_index_offset) {
             std::vector<radler::PsfOffset> offsets;
             if (py::len(py_psf_offsets)) {
               if (py_psf_offsets.ndim() != 2)
                 throw py::type_error(
                     "Non-empty PSF offsets must have two dimensions.");
               if (py_psf_offsets.shape(1) != 2)
                 throw py::type_error("PSF entries must have two values.");
               auto u = py_psf_offsets.unchecked<2>();
               for (py::ssize_t i = 0; i != py_psf_offsets.shape(0); ++i)
                 offsets.emplace_back(u(i, 0), u(i, 1));
             }
             return std::make_unique<radler::WorkTable>(
                 std::move(offsets), n_original_groups, n_deconvolution_groups,
                 channel_index_offset);
           }),
           py::arg("py_psf_offsets"), py::arg("n_original_groups"),
           py::arg("n_deconvolution_groups"), py::arg("channel_index_offset") = 0)
      .def_property_readonly("original_groups", [](const radler::WorkTable& t) {
        std::vector<std::vector<const radler::WorkTableEntry*>> g = t.OriginalGroups();
        return g;
      }, py::return_value_policy::reference_internal)
      .def_property_readonly("deconvolution_groups",
                             &radler::WorkTable::DeconvolutionGroups)
      .def("__len__", &radler::WorkTable::Size)
      .def("__str__", [](const radler::WorkTable& self) {
        std::stringstream s;
        s << self;
        return s.str();
      })
      .def_property_readonly("channel_index_offset",
                             &radler::WorkTable::GetChannelIndexOffset)
      .def("add_entry",
           [](radler::WorkTable& self, radler::WorkTableEntry& entry) {
             self.AddEntry(std::make_unique<radler::WorkTableEntry>(std::move(entry)));
           },
           py::arg("entry"))
      .def("__iter__",
           [](const radler::WorkTable& self) {
             return py::make_iterator(self.Begin(), self.End());
           },
           py::keep_alive<0, 1>());

  py::class_<radler::WorkTableEntry>(m, "WorkTableEntry")
      .def(py::init<>())
      .def_property_readonly("central_frequency",
                             &radler::WorkTableEntry::CentralFrequency)
      .def_readwrite("index", &radler::WorkTableEntry::index)
      .def_readwrite("band_start_frequency", &radler::WorkTableEntry::band_start_frequency)
      .def_readwrite("band_end_frequency", &radler::WorkTableEntry::band_end_frequency)
      .def_readwrite("polarization", &radler::WorkTableEntry::polarization)
      .def_readwrite("original_channel_index",
                     &radler::WorkTableEntry::original_channel_index)
      .def_readwrite("original_interval_index",
                     &radler::WorkTableEntry::original_interval_index)
      .def_readwrite("mask_channel_index", &radler::WorkTableEntry::mask_channel_index)
      .def_readwrite("image_weight", &radler::WorkTableEntry::image_weight)
      .def_property_readonly(
          "psfs",
          [](radler::WorkTableEntry& self) -> AccessorList& {
            return self.psf_accessors;
          },
          py::return_value_policy::reference)
      .def_property("residual", nullptr,
                    [](radler::WorkTableEntry& self, FloatArray& residual) {
                      self.residual_accessor =
                          MakeAccessor<radler::utils::LoadAndStoreImageAccessor>(residual);
                    })
      .def_property("model", nullptr,
                    [](radler::WorkTableEntry& self, FloatArray& model) {
                      self.model_accessor =
                          MakeAccessor<radler::utils::LoadAndStoreImageAccessor>(model);
                    });
}

void InitRadler(py::module& m) {  // python/pyradler.cc
  py::class_<radler::Radler>(m, "Radler")
      .def(py::init([](const radler::Settings& settings,
                       radler::WorkTable& work_table, double beam_size) {
             if (settings.thread_count == 0)
               throw std::runtime_error("Number of threads should be > 0.");
             return std::make_unique<radler::Radler>(
                 settings, std::make_unique<radler::WorkTable>(std::move(work_table)),
                 beam_size);
           }),
           py::arg("settings"), py::arg("work_table"), py::arg("beam_size"))
      .def(py::init([](const radler::Settings& settings, FloatArray& psf,
                       FloatArray& residual, FloatArray& model, double beam_size,
                       size_t n_deconvolution_groups, py::array_t<double>& frequencies,
                       py::array_t<double>& weights,
                       aocommon::PolarizationEnum polarization) {
             if (settings.thread_count == 0)
               throw std::runtime_error("Number of threads should be > 0.");
             if (psf.ndim() != residual.ndim() || psf.ndim() != model.ndim())
               throw std::runtime_error(
                   "Provided arrays should have equal dimension count.");
             for (py::ssize_t d = 0; d < psf.ndim(); ++d)
               if (residual.shape(d) != psf.shape(d) || model.shape(d) != psf.shape(d))
                 throw std::runtime_error("Provided arrays should have equal shape.");
             if (psf.ndim() != 2 && psf.ndim() != 3)
               throw std::runtime_error("Provided arrays should have 2 or 3 dimensions.");
             const size_t height = psf.shape(psf.ndim() - 2);
             const size_t width = psf.shape(psf.ndim() - 1);
             const size_t n_images = psf.ndim() == 2 ? 1 : psf.shape(0);
             if (settings.spectral_fitting.mode !=
                     schaapcommon::fitters::SpectralFittingMode::kNoFitting &&
                 frequencies.size() == 0)
               throw std::runtime_error(
                   "Frequencies are required when spectral fitting is enabled.");
             if (frequencies.size() > 0 &&
                 (frequencies.ndim() != 2 || size_t(frequencies.shape(0)) != n_images ||
                  frequencies.shape(1) != 2))
               throw std::runtime_error(
                   "Provided frequencies should have shape (n_images, 2).");
             if (weights.size() > 0 &&
                 (weights.ndim() != 1 || size_t(weights.shape(0)) != n_images))
               throw std::runtime_error("Provided weights should have shape (n_images).");
             auto table = std::make_unique<radler::WorkTable>(
                 std::vector<radler::PsfOffset>{}, n_images, n_deconvolution_groups);
             const size_t plane = width * height;
             for (size_t i = 0; i < n_images; ++i) {
               aocommon::Image p(psf.mutable_data() + i * plane, width, height);
               aocommon::Image r(residual.mutable_data() + i * plane, width, height);
               aocommon::Image mo(model.mutable_data() + i * plane, width, height);
               auto e = std::make_unique<radler::WorkTableEntry>();
               if (frequencies.size() > 0) {
                 auto u = frequencies.unchecked<2>();
                 e->band_start_frequency = u(i, 0);
                 e->band_end_frequency = u(i, 1);
               }
               e->polarization = polarization;
               e->original_channel_index = i;
               e->image_weight = weights.size() > 0 ? weights.unchecked<1>()(i) : 1.0;
               e->psf_accessors.emplace_back(
                   std::make_unique<radler::utils::LoadOnlyImageAccessor>(p));
               e->residual_accessor =
                   std::make_unique<radler::utils::LoadAndStoreImageAccessor>(r);
               e->model_accessor =
                   std::make_unique<radler::utils::LoadAndStoreImageAccessor>(mo);
               table->AddEntry(std::move(e));
             }
             return std::make_unique<radler::Radler>(settings, std::move(table),
                                                     beam_size);
           }),
           py::arg("settings"), py::arg("psf").noconvert(),
           py::arg("residual").noconvert(), py::arg("model").noconvert(),
           py::arg("beam_size"), py::arg("n_deconvolution_groups") = 0,
           py::arg("frequencies") = py::array_t<double>(),
           py::arg("weights") = py::array_t<double>(),
           py::arg("polarization") = aocommon::PolarizationEnum::StokesI)
      .def("perform",
           [](radler::Radler& self, size_t major_iteration_number) {
             py::gil_scoped_release release;
             bool another = false;
             self.Perform(another, major_iteration_number);
             return another;
           },
           py::arg("major_iteration_number"))
      .def("set_communicator", &radler::Radler::SetCommunicator, py::arg("communicator"))
      .def_property_readonly("iteration_number", &radler::Radler::IterationNumber)
      .def_property_readonly("component_list", &radler::Radler::GetComponentList);
}

void InitComponentList(py::module& m) {  // python/pycomponent_list.cc
  py::class_<radler::ComponentList>(m, "ComponentList")
      .def(py::init<>())
      .def(py::init<size_t, size_t, size_t, size_t>())
      .def_property("n_scales", &radler::ComponentList::NScales,
                    &radler::ComponentList::SetNScales)
      .def_property_readonly("n_frequencies", &radler::ComponentList::NFrequencies)
      .def("clear", &radler::ComponentList::Clear)
      .def_property_readonly("width", &radler::ComponentList::Width)
      .def_property_readonly("height", &radler::ComponentList::Height)
      .def("component_count", [](const radler::ComponentList& self, size_t s) {
        if (s >= self.NScales())
          throw std::out_of_range("Scale index out of range in component count");
        return self.ComponentCount(s);
      })
      .def("get_component",
           [](const radler::ComponentList& self, size_t s, size_t index) {
             // (x, y, values): ComponentList::GetComponent (component_list.h)
             if (s >= self.NScales() || index >= self.ComponentCount(s))
               throw std::out_of_range("Component index out of range");
             size_t x = 0, y = 0;
             std::vector<float> values(self.NFrequencies());
             self.GetComponent(s, index, x, y, values.data());
             return py::make_tuple(x, y, values);
           },
           py::arg("scale_index"), py::arg("index"))
      // C++ API members exposed for the restated cpp/test/test_component_list.cc
      .def("add",
           [](radler::ComponentList& self, size_t x, size_t y, size_t s,
              std::vector<float> values) {
             if (s >= self.NScales() || values.size() != self.NFrequencies())
               throw std::out_of_range("scale index or value count out of range");
             self.Add(x, y, s, values.data());
           },
           py::arg("x"), py::arg("y"), py::arg("scale_index"), py::arg("values"))
      .def("merge_duplicates", [](radler::ComponentList& self) { self.MergeDuplicates(); })
      .def("multiply_scale_component", &radler::ComponentList::MultiplyScaleComponent,
           py::arg("scale_index"), py::arg("position_index"), py::arg("channel"),
           py::arg("correction_factor"))
      .def("get_positions", [](const radler::ComponentList& self, size_t s) {
        if (s >= self.NScales()) throw std::out_of_range("Scale index out of range");
        py::list out;
        for (const auto& p : self.GetPositions(s)) out.append(py::make_tuple(p.x, p.y));
        return out;
      });
}

py::dict ResultDict(const radler::algorithms::ParallelDeconvolutionResult& r,
                    size_t iterations) {
  py::dict d;
  d["another_iteration_required"] = r.another_iteration_required;
  d["start_peak"] = r.start_peak ? py::cast(*r.start_peak) : py::none();
  d["end_peak"] = r.end_peak ? py::cast(*r.end_peak) : py::none();
  d["iterations"] = iterations;
  return d;
}

void InitTiling(py::module& m) {
  py::module t = m.def_submodule("tiling", "ParallelDeconvolution subimage geometry");
  t.def("make_subimages", [](py::array_t<float, py::array::c_style | py::array::forcecast> image,
                             size_t grid_w, size_t grid_h) {
    if (image.ndim() != 2) throw std::runtime_error("image must be 2-D");
    const size_t h = image.shape(0), w = image.shape(1);
    radler::Settings settings;
    settings.parallel.grid_width = grid_w;
    settings.parallel.grid_height = grid_h;
    std::vector<float> img(image.data(), image.data() + w * h);
    std::vector<size_t> psf_indices;
    const auto subs = radler::algorithms::MakeSubImages(img, w, h, nullptr, {}, settings,
                                                        psf_indices);
    py::array_t<uint32_t> boxes({py::ssize_t(subs.size()), py::ssize_t(4)});
    py::array_t<uint16_t> labels({py::ssize_t(h), py::ssize_t(w)});
    std::fill(labels.mutable_data(), labels.mutable_data() + w * h, 0);
    for (const auto& sub : subs) {
      uint32_t* b = boxes.mutable_data(py::ssize_t(sub.index), 0);
      b[0] = uint32_t(sub.x);
      b[1] = uint32_t(sub.y);
      b[2] = uint32_t(sub.width);
      b[3] = uint32_t(sub.height);
      for (size_t y = 0; y != sub.height; ++y)
        for (size_t x = 0; x != sub.width; ++x)
          if (sub.boundary_mask[y * sub.width + x])
            labels.mutable_data()[(y + sub.y) * w + x + sub.x] = uint16_t(sub.index + 1);
    }
    return py::make_tuple(boxes, labels);
  }, py::arg("image"), py::arg("grid_width"), py::arg("grid_height"));

  // math::DijkstraSplitter (cpp/math/dijkstra_splitter.h) member by member,
  // for the restated cpp/math/test/test_dijkstra_splitter.cc. Images are
  // C-contiguous float32 (h, w); outputs are modified in place.
  using F32 = py::array_t<float, py::array::c_style>;
  using B8 = py::array_t<bool, py::array::c_style>;
  auto splitter = [](const F32& image) {
    if (image.ndim() != 2) throw std::runtime_error("image must be 2-D");
    return radler::math::DijkstraSplitter(image.shape(1), image.shape(0));
  };
  t.def("divide_stats", [] {
    const radler::math::DivideStats st = radler::math::DijkstraSplitter::Stats();
    return py::make_tuple(st.key_order, st.exact, st.hybrid);
  }, "(key-order searches, exact heap-order searches, key-order paths completed from an "
     "exact prefix) run by this process");
  t.def("divide_vertically", [splitter](const F32& image, F32& output, size_t x1,
                                        size_t x2) {
    splitter(image).DivideVertically(image.data(), output.mutable_data(), x1, x2);
  });
  t.def("divide_horizontally", [splitter](const F32& image, F32& output, size_t y1,
                                          size_t y2) {
    splitter(image).DivideHorizontally(image.data(), output.mutable_data(), y1, y2);
  });
  t.def("add_vertical_divider", [splitter](const F32& image, F32& scratch, F32& output,
                                           size_t x1, size_t x2) {
    splitter(image).AddVerticalDivider(image.data(), scratch.mutable_data(),
                                       output.mutable_data(), x1, x2);
  });
  t.def("add_horizontal_divider", [splitter](const F32& image, F32& scratch, F32& output,
                                             size_t y1, size_t y2) {
    splitter(image).AddHorizontalDivider(image.data(), scratch.mutable_data(),
                                         output.mutable_data(), y1, y2);
  });
  t.def("flood_vertical_area", [splitter](const F32& division, size_t x, B8& mask) {
    size_t sx = 0, sw = 0;
    splitter(division).FloodVerticalArea(division.data(), x, mask.mutable_data(), sx, sw);
    return py::make_tuple(sx, sw);
  });
  t.def("flood_horizontal_area", [splitter](const F32& division, size_t y, B8& mask) {
    size_t sy = 0, sh = 0;
    splitter(division).FloodHorizontalArea(division.data(), y, mask.mutable_data(), sy,
                                           sh);
    return py::make_tuple(sy, sh);
  });
  t.def("get_bounding_mask", [](size_t width, size_t height, const B8& vertical_mask,
                                size_t vx, size_t vwidth, const B8& horizontal_mask,
                                B8& output) {
    size_t x = 0, y = 0, w = 0, h = 0;
    radler::math::DijkstraSplitter(width, height)
        .GetBoundingMask(vertical_mask.data(), vx, vwidth, horizontal_mask.data(),
                         output.mutable_data(), x, y, w, h);
    return py::make_tuple(x, y, w, h);
  });
}

void InitDistributed(py::module& m) {
  py::module d = m.def_submodule(
      "distributed",
      "Process-per-GPU split of ParallelDeconvolution (one rank per GPU)");
  py::class_<radler::Communicator, std::shared_ptr<radler::Communicator>>(d, "Communicator")
      .def_property_readonly("rank", &radler::Communicator::Rank)
      .def_property_readonly("size", &radler::Communicator::Size);
  py::class_<radler::RcclCommunicator, radler::Communicator,
             std::shared_ptr<radler::RcclCommunicator>>(d, "RcclCommunicator")
      .def(py::init([](int device, int size, int rank, py::bytes unique_id) {
             const std::string id = unique_id;
             if (id.size() != radler::RcclCommunicator::IdSize())
               throw std::runtime_error("RcclCommunicator: unique id has the wrong size");
             std::shared_ptr<radler::gpu::Session> session =
                 radler::gpu::Session::ForDevice(device);
             py::gil_scoped_release release;  // ncclCommInitRank blocks on the peers
             return std::make_shared<radler::RcclCommunicator>(session, size, rank,
                                                               id.data());
           }),
           py::arg("device"), py::arg("size"), py::arg("rank"), py::arg("unique_id"));
  d.def("rccl_id_size", &radler::RcclCommunicator::IdSize);
  d.def("rccl_unique_id", []() {
    std::string id(radler::RcclCommunicator::IdSize(), '\0');
    radler::RcclCommunicator::UniqueId(id.data());
    return py::bytes(id);
  });
  py::class_<radler::HostCommunicator, radler::Communicator,
             std::shared_ptr<radler::HostCommunicator>>(d, "HostCommunicator")
      .def(py::init([](int size, int rank, py::function broadcast, py::function max) {
             // the callbacks run while Perform has released the GIL
             auto bcast = [broadcast](void* data, size_t bytes, int root) {
               py::gil_scoped_acquire acquire;
               py::array_t<uint8_t> view({py::ssize_t(bytes)}, {py::ssize_t(1)},
                                         static_cast<uint8_t*>(data), py::none());
               broadcast(view, root);
             };
             auto fmax = [max](float v) {
               py::gil_scoped_acquire acquire;
               return max(v).cast<float>();
             };
             return std::make_shared<radler::HostCommunicator>(size, rank, bcast, fmax);
           }),
           py::arg("size"), py::arg("rank"), py::arg("broadcast"),
           py::arg("allreduce_max"),
           "Collectives on host memory supplied by the job: broadcast(uint8 array, "
           "root) fills the array in place on every rank but root; allreduce_max(x) "
           "returns the maximum over ranks")
      .def("broadcast_host",
           [](radler::HostCommunicator& self, py::array_t<uint8_t, py::array::c_style> a,
              int root) {
             self.BroadcastHost(a.mutable_data(), size_t(a.size()), root);
           },
           py::arg("array"), py::arg("root"))
      .def("allreduce_max",
           [](radler::HostCommunicator& self, float v) { return self.AllreduceMaxHost(v); },
           py::arg("value"));
  d.def("subimage_owner", &radler::SubImageOwner, py::arg("index"), py::arg("n_ranks"));
  d.def("lpt_owners", &radler::LptOwners, py::arg("costs"), py::arg("n_ranks"));
}

void InitGpu(py::module& m) {
  // utils::CalculateGoodFFTSize / GetConvolutionSize (fft_size_calculations.h:15-50)
  py::module u = m.def_submodule("utils", "FFT size helpers (host)");
  u.def("calculate_good_fft_size", &radler::utils::CalculateGoodFFTSize,
        py::arg("minimum_size"));
  u.def("get_convolution_size", &radler::utils::GetConvolutionSize, py::arg("scale"),
        py::arg("original_size"), py::arg("padding"));
  py::module g = m.def_submodule("gpu", "MI355X device helpers (bench/tests)");
  g.def("set_verbosity", &radler::log::SetVerbosity);
  // rdl_shutdown (rdl_hip.h): every device block, plan, stream and mapped
  // host buffer of the process released. Registered with Python's atexit,
  // which runs at interpreter finalization, before any C-level exit handler
  // (the HIP runtime's, a profiler's finalization); the C-level handler
  // librdl_hip registers itself stays as the fallback for C++ callers.
  // RDL_EXIT_SHUTDOWN=0 leaves teardown to the runtime.
  g.def("shutdown", []() { radler::gpu::Check(rdl_shutdown(), "rdl_shutdown"); });
  {
    const char* e = std::getenv("RDL_EXIT_SHUTDOWN");
    if (!(e && e[0] == '0'))
      py::module_::import("atexit").attr("register")(g.attr("shutdown"));
  }
  // RADLER_HOST_PROFILE=1 sections: {name: (count, total seconds)}
  g.def("host_profile", []() {
    py::dict out;
    for (const radler::prof::Entry& e : radler::prof::Snapshot())
      out[py::str(e.name)] = py::make_tuple(e.count, e.ns * 1e-9);
    return out;
  });
  g.def("host_profile_reset", &radler::prof::Reset);
  g.def("host_profile_enable", &radler::prof::SetEnabled, py::arg("on"));
  g.def(
      "local_rms",
      [](FloatArray integrated, int method, double window, double beam,
         double pixel_scale_x, double pixel_scale_y, double strength) {
        // Radler::Perform's local-RMS step on the device (cpp/radler.cc:196-216)
        if (integrated.ndim() != 2) throw std::runtime_error("expected a 2-D image");
        const size_t h = integrated.shape(0), w = integrated.shape(1), n = w * h;
        std::shared_ptr<radler::gpu::Session> session =
            radler::gpu::Session::ForDevice(radler::gpu::Session::DefaultDevice());
        radler::gpu::Session& s = *session;
        radler::gpu::Buffer in(s, n * sizeof(float)), rms(s, n * sizeof(float));
        s.H2D(in.Ptr(), integrated.data(), n * sizeof(float));
        py::array_t<float> out_rms({h, w}), out_factor({h, w});
        double lowest = 0.0;
        {
          py::gil_scoped_release release;
          if (method == 1)
            radler::math::rms_image::Make(s, rms.F(), in.F(), w, h, window, beam, beam,
                                          0.0, pixel_scale_x, pixel_scale_y);
          else
            radler::math::rms_image::MakeWithNegativityLimit(
                s, rms.F(), in.F(), w, h, window, beam, beam, 0.0, pixel_scale_x,
                pixel_scale_y);
          s.D2H(out_rms.mutable_data(), rms.F(), n * sizeof(float));
          lowest = radler::math::rms_image::MakeRmsFactorImage(s, rms.F(), n, strength);
          s.D2H(out_factor.mutable_data(), rms.F(), n * sizeof(float));
        }
        return py::make_tuple(out_rms, out_factor, lowest);
      },
      py::arg("integrated"), py::arg("method"), py::arg("window"), py::arg("beam"),
      py::arg("pixel_scale_x"), py::arg("pixel_scale_y"), py::arg("strength") = 1.0);
  // Settings::component_optimization_algorithm is C++-only in the reference's
  // bindings (python/pysettings.cc): set it through this helper so the
  // Settings attribute layout stays the reference's
  g.def(
      "set_component_optimization",
      [](radler::Settings& settings, radler::OptimizationAlgorithm algorithm) {
        settings.component_optimization_algorithm = algorithm;
      },
      py::arg("settings"), py::arg("algorithm"));
  g.def(
      "gradient_descent",
      [](FloatArray model, FloatArray residual, FloatArray psf) {
        // GenericClean's RunComponentOptimization for one image (padded 2W x 2H)
        if (model.ndim() != 2) throw std::runtime_error("expected 2-D images");
        const size_t h = model.shape(0), w = model.shape(1), n = w * h;
        if (size_t(residual.size()) != n || size_t(psf.size()) != n)
          throw std::runtime_error("image sizes differ");
        std::shared_ptr<radler::gpu::Session> session =
            radler::gpu::Session::ForDevice(radler::gpu::Session::DefaultDevice());
        radler::gpu::Session& s = *session;
        radler::gpu::Buffer dm(s, n * sizeof(float)), dr(s, n * sizeof(float)),
            dp(s, n * sizeof(float));
        s.H2D(dm.Ptr(), model.data(), n * sizeof(float));
        s.H2D(dr.Ptr(), residual.data(), n * sizeof(float));
        s.H2D(dp.Ptr(), psf.data(), n * sizeof(float));
        radler::math::GradientDescent(s, dm.F(), dr.F(), dp.F(), w, h, 2 * w, 2 * h);
        py::array_t<float> out({h, w});
        s.D2H(out.mutable_data(), dm.F(), n * sizeof(float));
        return out;
      },
      py::arg("model"), py::arg("residual"), py::arg("psf"));
  g.def(
      "linear_component_solve",
      [](FloatArray model, FloatArray residual, FloatArray psf) {
        // math::LinearComponentSolve(model, image, psf) (component_optimization.cc:258-263)
        if (model.ndim() != 2) throw std::runtime_error("expected 2-D images");
        const size_t h = model.shape(0), w = model.shape(1), n = w * h;
        if (size_t(residual.size()) != n || size_t(psf.size()) != n)
          throw std::runtime_error("image sizes differ");
        std::shared_ptr<radler::gpu::Session> session =
            radler::gpu::Session::ForDevice(radler::gpu::Session::DefaultDevice());
        radler::gpu::Session& s = *session;
        radler::gpu::Buffer dm(s, n * sizeof(float)), dr(s, n * sizeof(float)),
            dp(s, n * sizeof(float));
        s.H2D(dm.Ptr(), model.data(), n * sizeof(float));
        s.H2D(dr.Ptr(), residual.data(), n * sizeof(float));
        s.H2D(dp.Ptr(), psf.data(), n * sizeof(float));
        radler::math::LinearComponentSolve(s, dm.F(), dr.F(), dp.F(), w, h);
        py::array_t<float> out({h, w});
        s.D2H(out.mutable_data(), dm.F(), n * sizeof(float));
        return out;
      },
      py::arg("model"), py::arg("residual"), py::arg("psf"));
  g.def(
      "gradient_descent_with_variable_psf",
      [](std::vector<std::vector<std::pair<size_t, size_t>>> components, FloatArray image,
         std::vector<FloatArray> psfs, size_t padded_width, size_t padded_height) {
        // math::GradientDescentWithVariablePsf (component_optimization.cc:323-402)
        if (image.ndim() != 2) throw std::runtime_error("expected a 2-D image");
        const size_t h = image.shape(0), w = image.shape(1), n = w * h;
        if (psfs.size() != components.size())
          throw std::runtime_error("one PSF per component list is required");
        std::shared_ptr<radler::gpu::Session> session =
            radler::gpu::Session::ForDevice(radler::gpu::Session::DefaultDevice());
        radler::gpu::Session& s = *session;
        if (!padded_width) padded_width = 2 * w;
        if (!padded_height) padded_height = 2 * h;
        radler::gpu::Buffer di(s, n * sizeof(float)), dp(s, n * sizeof(float));
        s.H2D(di.Ptr(), image.data(), n * sizeof(float));
        std::vector<std::shared_ptr<radler::gpu::Buffer>> spectra;
        for (const FloatArray& p : psfs) {
          if (size_t(p.size()) != n) throw std::runtime_error("image sizes differ");
          s.H2D(dp.Ptr(), p.data(), n * sizeof(float));
          spectra.push_back(radler::algorithms::SubMinorLoop::MakePaddedPsfSpectrum(
              s, dp.F(), w, h, padded_width, padded_height));
        }
        std::vector<radler::gpu::Buffer> deltas = radler::math::GradientDescentWithVariablePsf(
            s, components, di.F(), spectra, w, h, padded_width, padded_height);
        py::list out;
        for (const radler::gpu::Buffer& d : deltas) {
          py::array_t<float> a({h, w});
          s.D2H(a.mutable_data(), d.F(), n * sizeof(float));
          out.append(a);
        }
        return out;
      },
      py::arg("components"), py::arg("image"), py::arg("psfs"), py::arg("padded_width") = 0,
      py::arg("padded_height") = 0);
  g.def(
      "make_rms_factor_image",
      [](FloatArray rms, double strength) {
        // math::rms_image::MakeRmsFactorImage (rms_image.cc:95-125)
        const size_t n = rms.size();
        std::shared_ptr<radler::gpu::Session> session =
            radler::gpu::Session::ForDevice(radler::gpu::Session::DefaultDevice());
        radler::gpu::Session& s = *session;
        radler::gpu::Buffer d(s, std::max<size_t>(n, 1) * sizeof(float));
        s.H2D(d.Ptr(), rms.data(), n * sizeof(float));
        const double lowest = radler::math::rms_image::MakeRmsFactorImage(s, d.F(), n, strength);
        py::array_t<float> out(n);
        s.D2H(out.mutable_data(), d.F(), n * sizeof(float));
        return py::make_tuple(out, lowest);
      },
      py::arg("rms"), py::arg("strength"));
  g.def(
      "ms_full_component_fitter",
      [](FloatArray residual, FloatArray model, FloatArray psf, std::vector<float> scales,
         std::vector<std::vector<std::pair<size_t, size_t>>> lists, double padding) {
        // MultiScaleAlgorithm::RunFullComponentFitter for one image
        const size_t h = residual.shape(0), w = residual.shape(1), n = w * h;
        std::shared_ptr<radler::gpu::Session> session =
            radler::gpu::Session::ForDevice(radler::gpu::Session::DefaultDevice());
        radler::gpu::Session& s = *session;
        radler::gpu::Buffer dr(s, n * sizeof(float)), dm(s, n * sizeof(float)),
            dp(s, n * sizeof(float));
        s.H2D(dr.Ptr(), residual.data(), n * sizeof(float));
        s.H2D(dm.Ptr(), model.data(), n * sizeof(float));
        s.H2D(dp.Ptr(), psf.data(), n * sizeof(float));
        radler::algorithms::multiscale::MultiScaleTransforms transforms(
            s, w, h, radler::MultiscaleShape::kTaperedQuadraticShape);
        const size_t pw = radler::utils::GetConvolutionSize(scales.back(), w, padding);
        const size_t ph = radler::utils::GetConvolutionSize(scales.back(), h, padding);
        radler::math::RunFullComponentFitter(s, dr.F(), dm.F(), dp.F(), w, h, scales, lists,
                                             transforms, pw, ph);
        py::array_t<float> out_r({h, w}), out_m({h, w});
        s.D2H(out_r.mutable_data(), dr.F(), n * sizeof(float));
        s.D2H(out_m.mutable_data(), dm.F(), n * sizeof(float));
        return py::make_tuple(out_r, out_m);
      },
      py::arg("residual"), py::arg("model"), py::arg("psf"), py::arg("scales"),
      py::arg("lists"), py::arg("padding") = 1.1);
  g.def(
      "ms_transform",
      [](FloatArray image, std::vector<float> scales, float max_scale, int shape) {
        // MultiScaleTransforms::Transform of one image per scale (the
        // transforms the multiscale algorithm runs, periodically extended
        // when the size is not FFT-friendly)
        if (image.ndim() != 2) throw std::runtime_error("expected a 2-D image");
        const size_t h = image.shape(0), w = image.shape(1), n = w * h;
        std::shared_ptr<radler::gpu::Session> session =
            radler::gpu::Session::ForDevice(radler::gpu::Session::DefaultDevice());
        radler::gpu::Session& s = *session;
        radler::algorithms::multiscale::MultiScaleTransforms transforms(
            s, w, h, radler::MultiscaleShape(shape));
        transforms.SetMaxScale(max_scale);
        radler::gpu::Buffer d(s, n * sizeof(float));
        py::array_t<float> out({py::ssize_t(scales.size()), py::ssize_t(h), py::ssize_t(w)});
        for (size_t i = 0; i != scales.size(); ++i) {
          s.H2D(d.Ptr(), image.data(), n * sizeof(float));
          transforms.Transform(d.F(), scales[i]);
          s.D2H(out.mutable_data(py::ssize_t(i)), d.F(), n * sizeof(float));
        }
        return py::make_tuple(out, transforms.PlaneWidth(), transforms.PlaneHeight());
      },
      py::arg("image"), py::arg("scales"), py::arg("max_scale"), py::arg("shape") = 0);
  g.def(
      "sliding_minimum",
      [](FloatArray image, size_t window) {
        if (image.ndim() != 2) throw std::runtime_error("expected a 2-D image");
        const size_t h = image.shape(0), w = image.shape(1), n = w * h;
        std::shared_ptr<radler::gpu::Session> session =
            radler::gpu::Session::ForDevice(radler::gpu::Session::DefaultDevice());
        radler::gpu::Session& s = *session;
        radler::gpu::Buffer in(s, n * sizeof(float)), out(s, n * sizeof(float)),
            scratch(s, 3 * n * sizeof(float));
        s.H2D(in.Ptr(), image.data(), n * sizeof(float));
        radler::math::rms_image::SlidingMinimum(s, out.F(), in.F(), scratch.F(), w, h,
                                                window);
        py::array_t<float> result({h, w});
        s.D2H(result.mutable_data(), out.F(), n * sizeof(float));
        return result;
      },
      py::arg("image"), py::arg("window"));
  // Radler::IterationNumber reports the first subimage's algorithm only
  // (cpp/radler.cc:406-408); bench.py counts the components of every
  // subimage of a gridded Perform
  g.def(
      "total_iteration_number",
      [](const radler::Radler& r) {
        if (!r.IsInitialized()) return size_t(0);
        const radler::algorithms::ParallelDeconvolution& p = r.Parallel();
        size_t total = 0;
        for (size_t i = 0; i != p.SubImageCount(); ++i)
          total += p.Algorithm(i).IterationNumber();
        return total;
      },
      py::arg("radler"));
  // The device-resident ImageSet (cpp/image_set.h) for the restated
  // cpp/test/test_image_set.cc: planes set/read through host copies, the
  // integrations and averaging run on the device.
  struct PyImageSet {
    std::shared_ptr<radler::gpu::Session> session;
    std::unique_ptr<radler::ImageSet> set;
    py::array_t<float> Plane(const float* d) const {
      py::array_t<float> out({py::ssize_t(set->Height()), py::ssize_t(set->Width())});
      session->D2H(out.mutable_data(), d, set->PlaneSize() * sizeof(float));
      return out;
    }
  };
  py::class_<PyImageSet>(g, "ImageSet")
      .def(py::init([](const radler::WorkTable& table, bool squared_joins,
                       const std::set<aocommon::PolarizationEnum>& linked, size_t width,
                       size_t height) {
             auto p = std::make_unique<PyImageSet>();
             p->session = radler::gpu::Session::ForDevice(radler::gpu::Session::DefaultDevice());
             p->set = std::make_unique<radler::ImageSet>(table, squared_joins, linked, width,
                                                         height, *p->session);
             return p;
           }),
           py::arg("work_table"), py::arg("squared_joins"), py::arg("linked_polarizations"),
           py::arg("width"), py::arg("height"), py::keep_alive<1, 2>())
      .def_property_readonly("n_original_channels",
                             [](const PyImageSet& s) { return s.set->NOriginalChannels(); })
      .def_property_readonly("n_deconvolution_channels",
                             [](const PyImageSet& s) { return s.set->NDeconvolutionChannels(); })
      .def_property_readonly("psf_count", [](const PyImageSet& s) { return s.set->PsfCount(); })
      .def_property_readonly("square_joined_channels",
                             [](const PyImageSet& s) { return s.set->SquareJoinedChannels(); })
      .def("__len__", [](const PyImageSet& s) { return s.set->Size(); })
      .def("psf_index", [](const PyImageSet& s, size_t i) { return s.set->PsfIndex(i); })
      .def("fill_zero", [](PyImageSet& s) { s.set->Fill(0.0f); })
      .def("set_image",
           [](PyImageSet& s, size_t i, FloatArray image) {
             if (i >= s.set->Size() || size_t(image.size()) != s.set->PlaneSize())
               throw std::out_of_range("set_image: index or size out of range");
             s.session->H2D(s.set->Data(i), image.data(), s.set->PlaneSize() * sizeof(float));
           })
      .def("image", [](const PyImageSet& s, size_t i) {
        if (i >= s.set->Size()) throw std::out_of_range("image index out of range");
        return s.Plane(s.set->Data(i));
      })
      .def("linear_integrated", [](const PyImageSet& s) {
        radler::gpu::Buffer d(*s.session, s.set->PlaneSize() * sizeof(float));
        s.set->GetLinearIntegrated(d.F());
        return s.Plane(d.F());
      })
      .def("square_integrated", [](const PyImageSet& s) {
        radler::gpu::Buffer d(*s.session, s.set->PlaneSize() * sizeof(float));
        s.set->GetSquareIntegrated(d.F());
        return s.Plane(d.F());
      })
      .def("load_and_average", [](PyImageSet& s, bool use_residual_images) {
        s.set->LoadAndAverage(use_residual_images);
      }, py::arg("use_residual_images"))
      .def("load_and_average_psfs", [](const PyImageSet& s) {
        // [psf index][deconvolution channel] -> 2-D arrays
        py::list out;
        for (const radler::gpu::Planes& planes : s.set->LoadAndAveragePsfs()) {
          py::list channels;
          for (size_t ch = 0; ch != planes.count; ++ch) {
            py::array_t<float> a({py::ssize_t(planes.height), py::ssize_t(planes.width)});
            s.session->D2H(a.mutable_data(), planes.Plane(ch),
                           planes.PlaneSize() * sizeof(float));
            channels.append(a);
          }
          out.append(channels);
        }
        return out;
      })
      .def("interpolate_and_store_model",
           [](PyImageSet& s, const schaapcommon::fitters::SpectralFitter* fitter) {
             s.set->InterpolateAndStoreModel(fitter);
           },
           py::arg("fitter") = nullptr)
      .def("assign_and_store_residual", [](PyImageSet& s) { s.set->AssignAndStoreResidual(); });
  py::class_<radler::DeviceRun>(g, "DeviceRun")
      .def(py::init([](const radler::Settings& settings, FloatArray psf,
                       FloatArray residual, std::vector<double> weights,
                       double beam_size, bool trace) {
             const size_t n = psf.ndim() == 2 ? 1 : psf.shape(0);
             return std::make_unique<radler::DeviceRun>(
                 settings, psf.data(), residual.data(), n, weights, beam_size, trace);
           }),
           py::arg("settings"), py::arg("psf"), py::arg("residual"),
           py::arg("weights") = std::vector<double>(), py::arg("beam_size") = 0.0,
           py::arg("trace") = true)
      .def("restore", &radler::DeviceRun::Restore)
      .def("set_communicator", &radler::DeviceRun::SetCommunicator,
           py::arg("communicator"))
      .def("set_rms_factor",
           [](radler::DeviceRun& self, const std::vector<float>& factor) {
             self.SetRmsFactorImage(factor);
           },
           py::arg("factor"))
      .def("execute",
           [](radler::DeviceRun& self) {
             radler::algorithms::ParallelDeconvolutionResult r;
             {
               py::gil_scoped_release release;
               r = self.Execute();
             }
             return ResultDict(r, self.LastIterations());
           })
      .def("sync", &radler::DeviceRun::Sync)
      .def("residual", [](const radler::DeviceRun& self) {
        std::vector<float> v = self.Residual();
        return py::array_t<float>(v.size(), v.data());
      })
      .def("model", [](const radler::DeviceRun& self) {
        std::vector<float> v = self.Model();
        return py::array_t<float>(v.size(), v.data());
      })
      .def("trace", [](const radler::DeviceRun& self, size_t index) {
        const std::vector<uint32_t>& t = self.Trace(index);
        py::array_t<uint32_t> a({py::ssize_t(t.size() / 3), py::ssize_t(3)});
        std::copy(t.begin(), t.end(), a.mutable_data());
        return a;
      }, py::arg("index") = 0)
      .def("iuwt_steps", [](const radler::DeviceRun& self, size_t index) {
        // (succeeded, scale, x, y, end_scale, min_scale, area, max_value,
        //  trimmed_width)
        py::list out;
        for (const auto& s : self.IuwtSteps(index))
          out.append(py::make_tuple(s.succeeded, s.scale, s.x, s.y, s.end_scale,
                                    s.min_scale, s.area, s.max_value, s.trimmed_width));
        return out;
      }, py::arg("index") = 0)
      .def("clean_owners", [](const radler::DeviceRun& self) { return self.CleanOwners(); })
      .def("subimages", [](const radler::DeviceRun& self, size_t width, size_t height) {
        // (boxes [n][x, y, w, h], labels [h][w]: subimage index + 1 inside its
        // boundary mask)
        const auto& subs = self.SubImages();
        py::array_t<uint32_t> boxes({py::ssize_t(subs.size()), py::ssize_t(4)});
        py::array_t<uint16_t> labels({py::ssize_t(height), py::ssize_t(width)});
        std::fill(labels.mutable_data(), labels.mutable_data() + width * height, 0);
        for (const auto& sub : subs) {
          uint32_t* b = boxes.mutable_data(py::ssize_t(sub.index), 0);
          b[0] = uint32_t(sub.x);
          b[1] = uint32_t(sub.y);
          b[2] = uint32_t(sub.width);
          b[3] = uint32_t(sub.height);
          for (size_t y = 0; y != sub.height; ++y)
            for (size_t x = 0; x != sub.width; ++x)
              if (sub.boundary_mask[y * sub.width + x])
                labels.mutable_data()[(y + sub.y) * width + x + sub.x] =
                    uint16_t(sub.index + 1);
        }
        return py::make_tuple(boxes, labels);
      }, py::arg("width"), py::arg("height"))
      .def("session_handle", [](radler::DeviceRun& self) {
        return reinterpret_cast<uintptr_t>(self.Session().Handle());
      })
      .def("stream_handle", [](radler::DeviceRun& self) {
        return reinterpret_cast<uintptr_t>(rdl_session_stream(self.Session().Handle()));
      });
}

}  // namespace

PYBIND11_MODULE(radler, m) {  // python/pywrappers.cc
  m.doc() = "MI355X-native Radio Astronomical Deconvolution Library (radler API)";
  InitSettings(m);
  InitWorkTable(m);
  InitSpectralFitter(m);
  InitRadler(m);
  InitComponentList(m);
  InitGpu(m);
  InitTiling(m);
  InitDistributed(m);
}
