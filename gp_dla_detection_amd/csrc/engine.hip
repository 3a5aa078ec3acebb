// C-ABI of libgpdla.so (include/gpdla.h): engine lifecycle, device workspaces, batching,
// kernel-time accounting and the standalone voigt / log_mvnpdf_low_rank entry points.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gpdla.h"
#include "internal.h"

using namespace gpdla;

namespace {
thread_local std::string g_last_error;
thread_local LaunchTimes g_launch_times;
}  // namespace

namespace gpdla {

int set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

LaunchTimes& launch_times() { return g_launch_times; }

int check_device(int32_t device) {
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count == 0)
    return set_error(GPDLA_EDEVICE, "no HIP device available (%s): libgpdla has no CPU fallback",
                     hipGetErrorString(e));
  if (device < 0 || device >= count)
    return set_error(GPDLA_EINVAL, "device %d out of range (%d devices)", device, count);
  return GPDLA_OK;
}

}  // namespace gpdla

namespace {

// ---- line-profile data (fitted once per process on the host; layout in internal.h)
struct HostLineData {
  std::vector<double> buf;
};

const HostLineData& host_line_data() {
  static HostLineData d;
  static std::once_flag once;
  std::call_once(once, [] {
    d.buf.assign(kLineBufDoubles, 0.0);
    for (int j = 0; j < kMaxLines; ++j) {
      fit_core_table(j, d.buf.data() + (size_t)j * kCoreTable);
      fit_wing_line(j, d.buf.data() + kLineBufWing + (size_t)j * kWingStride);
    }
    for (int j = 0; j < kMaxLines; ++j) {
      // fac_j = c / (lambda_j 1e8) / (sigma sqrt 2): x_j = lambda fac_j / (1+z) - c / (sigma sqrt 2)
      const long double f = (long double)kCcgs / ((long double)kTransitionWavelengths[j] * 1e8L) /
                            ((long double)kSigma * std::sqrt(2.0L));
      d.buf[kLineBufFac + j] = (double)f;
    }
    for (int j = 0; j < 64; ++j) d.buf[kLineBufExp2 + j] = (double)std::exp2((long double)j / 64.0L);
    for (int j = 0; j < 128; ++j) d.buf[kLineBufExp128 + j] = (double)std::exp2((long double)j / 128.0L);
  });
  return d;
}

LineArgs make_line_args(const double* d_buf) {
  LineArgs l{};
  l.buf = d_buf;
  return l;
}

template <class T>
int grow(T** p, size_t* cap, size_t count) {
  if (count <= *cap && *p) return GPDLA_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  size_t want = std::max<size_t>(count, 1);
  HIP_TRY(hipMalloc((void**)p, want * sizeof(T)));
  *cap = want;
  return GPDLA_OK;
}

struct TimedLaunch {
  hipEvent_t start, stop;
  int kind;  // 0 prep, 1 likelihood, 2 reduce, 3 contraction (panel-GEMM paths, inside 1)
};

// One of the two staging sets of the host-buffer pipeline (gpdla_engine_process with host inputs
// and host results): the batch's inputs and results on the device, and the events that order the
// copy stream against the compute stream.
struct HostStage {
  double *wl = nullptr, *flux = nullptr, *noise = nullptr, *z = nullptr;
  uint8_t* mask = nullptr;
  double *sll = nullptr, *llnull = nullptr, *lldla = nullptr, *zmin = nullptr, *zmax = nullptr;
  int32_t* npix = nullptr;
  size_t cap_wl = 0, cap_flux = 0, cap_noise = 0, cap_mask = 0, cap_z = 0, cap_sll = 0;
  size_t cap_o[5] = {0, 0, 0, 0, 0};
  hipEvent_t in_ready = nullptr;   // copy stream: this batch's inputs are on the device
  hipEvent_t in_free = nullptr;    // compute stream: prep_kernel has read them
  hipEvent_t out_ready = nullptr;  // compute stream: the batch's results are written
  hipEvent_t out_free = nullptr;   // copy stream: they are back on the host
};

}  // namespace

struct gpdla_engine {
  int device = 0;
  int K = 0;
  int64_t S = 0;
  bool gemm = false;                 // panel-GEMM path (gemm_path.hip + gemm_f64 / gemm_i8) instead of fused
  bool i8 = false;                   // fused path with the int8 Ozaki contraction (kernels_i8.hip)
  int i8_nd = 4;                     // int8 panel-GEMM digit planes: 4 (levels <= 3) or 3 (_I8_24)
  gpdla_params params{};
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;

  // resident model / samples / line data
  double *d_rest = nullptr, *d_mu = nullptr, *d_M = nullptr, *d_logom = nullptr;
  int32_t num_rest = 0;
  double c0 = 0, tau0 = 0, beta = 0;
  int32_t om2_hi_e = 0;  // binary exponent of max omega^2 (1 + c_0)^2 over the rest grid (prep units)
  double *d_off = nullptr, *d_nhi = nullptr;  // samples in ascending-offset (z_DLA) order
  int32_t* d_perm = nullptr;                   // sorted sample index -> caller's sample index
  double* d_lines = nullptr;
  int32_t* d_status = nullptr;

  // batch workspaces
  size_t cap_meta = 0, cap_q = 0, cap_slots = 0, cap_lam = 0, cap_sll = 0, cap_scr = 0;
  size_t cap_smap = 0, cap_wl = 0, cap_flux = 0, cap_noise = 0, cap_mask = 0, cap_z = 0;
  int64_t* d_meta = nullptr;  // [offsets(Q+1) | slot_base | lam_base | slot_cap]
  double *d_wl = nullptr, *d_flux = nullptr, *d_noise = nullptr;
  uint8_t* d_mask = nullptr;
  double* d_z = nullptr;
  SpecInfo* d_info = nullptr;
  double *d_panel = nullptr, *d_lam = nullptr;
  int32_t* d_smap = nullptr;
  double* d_scratch = nullptr;
  double *d_sll = nullptr, *d_llnull = nullptr, *d_lldla = nullptr, *d_zmin = nullptr,
         *d_zmax = nullptr;
  int32_t* d_npix = nullptr;
  size_t cap_qout = 0;
  // panel-GEMM path workspaces
  double *d_pm = nullptr, *d_srow = nullptr, *d_wg = nullptr, *d_wu = nullptr, *d_G = nullptr,
         *d_U = nullptr, *d_q1p = nullptr, *d_ldp = nullptr;
  size_t cap_pm = 0, cap_srow = 0, cap_wg = 0, cap_wu = 0, cap_G = 0, cap_U = 0, cap_q1p = 0,
         cap_ldp = 0;
  // int8 fused path workspaces
  uint8_t* d_pi8 = nullptr;          // fused: digit chunks; panel-GEMM: B digit planes per spectrum
  uint8_t* d_ai8 = nullptr;          // panel-GEMM int8: A digit planes of a sample chunk
  size_t cap_ai8 = 0;
  double *d_psc = nullptr, *d_pent = nullptr;
  size_t cap_pi8 = 0, cap_psc = 0, cap_pent = 0;

  // host-buffer pipeline: batch b's results are copied back, and batch b + 1's inputs copied in, on
  // copy_stream while batch b + 1 (resp. b) computes; the two stages alternate
  HostStage hs[2];
  hipStream_t copy_stream = nullptr;
  // the panel-GEMM paths' extra compute streams (panel_streams > 1): spectrum q of a batch runs on
  // stream q % panel_streams (0 = the engine's stream) with its own workspace set, so one spectrum's
  // kernels fill the last-round tails of the others'
  static constexpr int kMaxPanelStreams = 4;
  int panel_streams = 2;
  hipStream_t panel_stream[kMaxPanelStreams] = {};
  hipEvent_t panel_fork = nullptr, panel_join[kMaxPanelStreams] = {};
  int64_t ws_ai8 = 0, ws_G = 0, ws_U = 0, ws_wp = 0, ws_w = 0;  // per-set workspace sizes (bytes / doubles)

  // pinned host metadata (reused after meta_ready completes)
  int64_t* h_meta = nullptr;
  size_t cap_hmeta = 0;
  hipEvent_t meta_done = nullptr;


  std::vector<TimedLaunch> pending;
  gpdla_stats stats{};
};

namespace {

int record_start(gpdla_engine* e, TimedLaunch* t, int kind, hipStream_t s = nullptr) {
  HIP_TRY(hipEventCreate(&t->start));
  HIP_TRY(hipEventCreate(&t->stop));
  t->kind = kind;
  HIP_TRY(hipEventRecord(t->start, s ? s : e->stream));
  return GPDLA_OK;
}

int resolve_events(gpdla_engine* e) {
  for (auto& t : e->pending) {
    HIP_TRY(hipEventSynchronize(t.stop));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, t.start, t.stop));
    if (t.kind == 0) { e->stats.prep_ms += ms; e->stats.prep_launches++; }
    if (t.kind == 1) { e->stats.likelihood_ms += ms; e->stats.likelihood_launches++; }
    if (t.kind == 2) { e->stats.reduce_ms += ms; e->stats.reduce_launches++; }
    if (t.kind == 3) { e->stats.contraction_ms += ms; e->stats.contraction_launches++; }
    (void)hipEventDestroy(t.start);
    (void)hipEventDestroy(t.stop);
  }
  e->pending.clear();
  return GPDLA_OK;
}

int validate_params(const gpdla_params* p) {
  if (p->num_lines < 1 || p->num_lines > kMaxLines)
    return set_error(GPDLA_EINVAL, "num_lines=%d outside [1, %d] (voigt.c:16)", p->num_lines, kMaxLines);
  if (p->width != kWidth)
    return set_error(GPDLA_EINVAL, "width=%d but the instrument profile is compiled for %d (voigt.c:229)",
                     p->width, kWidth);
  if (p->absorption_mode != GPDLA_ABSORPTION_REFERENCE && p->absorption_mode != GPDLA_ABSORPTION_UNMASKED)
    return set_error(GPDLA_EINVAL, "absorption_mode=%d", p->absorption_mode);
  if (!(p->max_lambda > p->min_lambda) || !(p->pixel_spacing > 0) || !(p->lya_wavelength > 0))
    return set_error(GPDLA_EINVAL, "invalid wavelength parameters");
  if (p->max_batch_spectra < 0) return set_error(GPDLA_EINVAL, "max_batch_spectra < 0");
  if (p->path != GPDLA_PATH_AUTO && p->path != GPDLA_PATH_FUSED && p->path != GPDLA_PATH_PANEL_GEMM &&
      p->path != GPDLA_PATH_FUSED_I8 && p->path != GPDLA_PATH_PANEL_GEMM_I8 && p->path != GPDLA_PATH_PANEL_GEMM_I8_24)
    return set_error(GPDLA_EINVAL, "path=%d", p->path);
  return GPDLA_OK;
}

int upload(void* dst, const void* src, size_t bytes, hipStream_t s) {
  HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
  return GPDLA_OK;
}

}  // namespace

extern "C" {

int32_t gpdla_version(void) { return GPDLA_ABI_VERSION; }

int gpdla_last_call_kernel_ms(double* ms, int32_t capacity, int32_t* count) {
  if (!count || capacity < 0 || (capacity > 0 && !ms))
    return set_error(GPDLA_EINVAL, "last_call_kernel_ms: null argument or negative capacity");
  const LaunchTimes& t = launch_times();
  *count = t.done;
  for (int i = 0; i < t.done && i < capacity; ++i) ms[i] = t.ms[i];
  return GPDLA_OK;
}

int32_t gpdla_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

int gpdla_device_pci_bus_id(int32_t device, char* buf, int32_t len) {
  if (!buf || len < 13) return set_error(GPDLA_EINVAL, "pci bus id buffer needs >= 13 bytes");
  int c = gpdla_device_count();
  if (c == 0) return set_error(GPDLA_EDEVICE, "no HIP device");
  if (device < 0 || device >= c) return set_error(GPDLA_EINVAL, "device %d outside [0, %d)", device, c);
  HIP_TRY(hipDeviceGetPCIBusId(buf, len, device));
  return GPDLA_OK;
}

const char* gpdla_last_error(void) { return g_last_error.c_str(); }

int gpdla_diag_faddeeva_w(double x, double y, double* re, double* im);  // faddeeva_host.cpp

int gpdla_diag_line_table_error(int32_t line, double* max_rel_err) {
  if (line < 0 || line >= kMaxLines || !max_rel_err) return set_error(GPDLA_EINVAL, "bad line");
  *max_rel_err = line_profile_error(line);  // core, wing and outer wing
  return GPDLA_OK;
}

void gpdla_engine_destroy(gpdla_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  (void)hipStreamSynchronize(e->stream);  // (the null stream too)
  if (e->copy_stream) (void)hipStreamSynchronize(e->copy_stream);
  for (auto& t : e->pending) { (void)hipEventDestroy(t.start); (void)hipEventDestroy(t.stop); }
  for (HostStage& h : e->hs) {
    void* hb[] = {h.wl, h.flux, h.noise, h.z, h.mask, h.sll, h.llnull, h.lldla, h.zmin, h.zmax, h.npix};
    for (void* b : hb)
      if (b) (void)hipFree(b);
    for (hipEvent_t ev : {h.in_ready, h.in_free, h.out_ready, h.out_free})
      if (ev) (void)hipEventDestroy(ev);
  }
  if (e->copy_stream) (void)hipStreamDestroy(e->copy_stream);
  for (int i = 1; i < gpdla_engine::kMaxPanelStreams; ++i) {
    if (e->panel_stream[i]) {
      (void)hipStreamSynchronize(e->panel_stream[i]);
      (void)hipStreamDestroy(e->panel_stream[i]);
    }
    if (e->panel_join[i]) (void)hipEventDestroy(e->panel_join[i]);
  }
  if (e->panel_fork) (void)hipEventDestroy(e->panel_fork);
  void* bufs[] = {e->d_rest, e->d_mu, e->d_M, e->d_logom, e->d_off, e->d_nhi, e->d_perm, e->d_lines,
                  e->d_status, e->d_meta, e->d_wl, e->d_flux, e->d_noise, e->d_mask, e->d_z,
                  e->d_info, e->d_panel, e->d_lam, e->d_smap, e->d_scratch, e->d_sll,
                  e->d_llnull, e->d_lldla, e->d_zmin, e->d_zmax, e->d_npix, e->d_pm, e->d_srow,
                  e->d_wg, e->d_wu, e->d_G, e->d_U, e->d_q1p, e->d_ldp, e->d_pi8, e->d_psc,
                  e->d_pent, e->d_ai8};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (e->h_meta) (void)hipHostFree(e->h_meta);
  if (e->meta_done) (void)hipEventDestroy(e->meta_done);

  if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
  delete e;
}

int gpdla_engine_create(int32_t device, const gpdla_model* model, const gpdla_samples* samples,
                        const gpdla_params* params, gpdla_engine** out) {
  if (!model || !samples || !params || !out) return set_error(GPDLA_EINVAL, "null argument");
  *out = nullptr;
  int rc = check_device(device);
  if (rc) return rc;
  if ((rc = validate_params(params))) return rc;
  // fused paths: a rank between the compiled ones runs on the next compiled rank, M zero-padded
  // (fused_rank, kernels.hip: exact)
  const int k_fused = fused_rank(model->k), k_i8 = i8_fused_rank(model->k);
  const bool fused_ok = k_fused > 0;
  const bool gemm_i8 = params->path == GPDLA_PATH_PANEL_GEMM_I8 || params->path == GPDLA_PATH_PANEL_GEMM_I8_24;
  const bool use_gemm = params->path == GPDLA_PATH_PANEL_GEMM || gemm_i8 ||
                        (params->path == GPDLA_PATH_AUTO && !fused_ok);
  const bool use_i8 = params->path == GPDLA_PATH_FUSED_I8 || gemm_i8;
  if (gemm_i8 && params->num_lines != 3)
    return set_error(GPDLA_EUNSUPPORTED, "int8 panel-GEMM path needs num_lines=3 (num_lines=%d)", params->num_lines);
  if (params->path == GPDLA_PATH_FUSED_I8 && (k_i8 == 0 || params->num_lines != 3))
    return set_error(GPDLA_EUNSUPPORTED, "int8 fused path needs k<=20 and num_lines=3 (k=%d, num_lines=%d)",
                     model->k, params->num_lines);
  if (!use_gemm && !fused_ok)
    return set_error(GPDLA_EUNSUPPORTED, "rank k=%d above the fused path's compiled ranks (<= 24)", model->k);
  if (use_gemm && (model->k < 1 || model->k > kGemmMaxK))
    return set_error(GPDLA_EUNSUPPORTED, "rank k=%d outside the panel-GEMM path's 1..%d", model->k, kGemmMaxK);
  if (model->num_rest < 2 || !model->rest_wavelengths || !model->mu || !model->M || !model->log_omega)
    return set_error(GPDLA_EINVAL, "invalid model");
  for (int i = 1; i < model->num_rest; ++i)
    if (!(model->rest_wavelengths[i] > model->rest_wavelengths[i - 1]))
      return set_error(GPDLA_EINVAL, "rest_wavelengths must be strictly increasing");
  if (samples->num_samples < 1 || !samples->offset_samples || !samples->nhi_samples)
    return set_error(GPDLA_EINVAL, "invalid samples");
  // column densities: the sweeps' exp needs N >= 0 and finite (kernels.hip likelihood_kernel bounds
  // N tot by them); generate_dla_samples.m:20-53 only produces positive N_HI
  for (int64_t i = 0; i < samples->num_samples; ++i)
    if (!(samples->nhi_samples[i] >= 0.0 && samples->nhi_samples[i] < INFINITY))
      return set_error(GPDLA_EINVAL, "nhi_samples[%lld] = %g: column densities must be finite and >= 0",
                       (long long)i, samples->nhi_samples[i]);

  HIP_TRY(hipSetDevice(device));
  gpdla_engine* e = new gpdla_engine();
  e->device = device;
  e->K = use_gemm ? model->k : (use_i8 ? k_i8 : k_fused);  // the rank the kernels run at
  e->S = samples->num_samples;
  e->gemm = use_gemm;
  e->i8 = use_i8;
  e->i8_nd = params->path == GPDLA_PATH_PANEL_GEMM_I8_24 ? 3 : 4;
  e->params = *params;
  e->num_rest = model->num_rest;
  e->c0 = std::exp(model->log_c_0);     // process_qsos.m:84-86
  e->tau0 = std::exp(model->log_tau_0);
  e->beta = std::exp(model->log_beta);
  {  // omega^2 = exp(2 log omega) sf^2 with sf = 1 - exp(-tau_0 (1 + z)^beta) + c_0 in [c_0, 1 + c_0]
    double lo_max = -INFINITY;
    for (int i = 0; i < model->num_rest; ++i) lo_max = std::max(lo_max, model->log_omega[i]);
    const double om2_max = std::exp(2 * lo_max) * (1 + e->c0) * (1 + e->c0);
    e->om2_hi_e = (om2_max > 0 && om2_max < INFINITY) ? (int32_t)std::ilogb(om2_max) : 0;
  }
  auto fail = [&](int code) { gpdla_engine_destroy(e); return code; };
#define TRY_E(x) do { int r_ = (x); if (r_) return fail(r_); } while (0)
  if (hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking) != hipSuccess)
    return fail(set_error(GPDLA_EDEVICE, "hipStreamCreate failed"));
  e->stream = e->own_stream;
  if (hipEventCreateWithFlags(&e->meta_done, hipEventDisableTiming) != hipSuccess)
    return fail(set_error(GPDLA_EDEVICE, "hipEventCreate failed"));


  const size_t G = model->num_rest, K = e->K, k_model = model->k;
  std::vector<double> Mrow(G * K, 0.0);  // columns k_model..K-1: the fused paths' zero padding
  for (size_t g = 0; g < G; ++g)
    for (size_t c = 0; c < k_model; ++c) Mrow[g * K + c] = model->M[g + c * G];  // col-major -> row-major
  size_t dummy = 0;
  TRY_E(grow(&e->d_rest, &dummy, G)); dummy = 0;
  TRY_E(grow(&e->d_mu, &dummy, G)); dummy = 0;
  TRY_E(grow(&e->d_M, &dummy, G * K)); dummy = 0;
  TRY_E(grow(&e->d_logom, &dummy, G)); dummy = 0;
  TRY_E(grow(&e->d_off, &dummy, (size_t)e->S)); dummy = 0;
  TRY_E(grow(&e->d_nhi, &dummy, (size_t)e->S)); dummy = 0;
  TRY_E(grow(&e->d_perm, &dummy, (size_t)e->S)); dummy = 0;
  const std::vector<double>& lines = host_line_data().buf;
  TRY_E(grow(&e->d_lines, &dummy, lines.size())); dummy = 0;
  TRY_E(grow(&e->d_status, &dummy, 1));
  TRY_E(upload(e->d_rest, model->rest_wavelengths, G * 8, e->stream));
  TRY_E(upload(e->d_mu, model->mu, G * 8, e->stream));
  TRY_E(upload(e->d_M, Mrow.data(), G * K * 8, e->stream));
  TRY_E(upload(e->d_logom, model->log_omega, G * 8, e->stream));
  // Samples are swept in ascending offset order: z_DLA = zmin + (zmax - zmin) offset is then
  // ascending for every spectrum, so the 16 samples of a wave put their line centres on nearly
  // the same pixels and the divergent |x| < kCoreX branch is taken in few steps.  Each sample's
  // arithmetic is lane-independent, so results are unchanged; outputs scatter back via d_perm.
  std::vector<int32_t> perm((size_t)e->S);
  for (int64_t i = 0; i < e->S; ++i) perm[i] = (int32_t)i;
  std::stable_sort(perm.begin(), perm.end(), [&](int32_t a, int32_t b) {
    return samples->offset_samples[a] < samples->offset_samples[b];
  });
  std::vector<double> off_sorted((size_t)e->S), nhi_sorted((size_t)e->S);
  for (int64_t i = 0; i < e->S; ++i) {
    off_sorted[i] = samples->offset_samples[perm[i]];
    nhi_sorted[i] = samples->nhi_samples[perm[i]];
  }
  TRY_E(upload(e->d_off, off_sorted.data(), (size_t)e->S * 8, e->stream));
  TRY_E(upload(e->d_nhi, nhi_sorted.data(), (size_t)e->S * 8, e->stream));
  TRY_E(upload(e->d_perm, perm.data(), (size_t)e->S * 4, e->stream));
  TRY_E(upload(e->d_lines, lines.data(), lines.size() * 8, e->stream));
  if (hipMemsetAsync(e->d_status, 0, 4, e->stream) != hipSuccess ||
      hipStreamSynchronize(e->stream) != hipSuccess)
    return fail(set_error(GPDLA_EDEVICE, "engine upload failed"));
#undef TRY_E
  *out = e;
  return GPDLA_OK;
}

int gpdla_engine_set_stream(gpdla_engine* e, void* hip_stream) {
  if (!e) return set_error(GPDLA_EINVAL, "null engine");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->stream = hip_stream ? (hipStream_t)hip_stream : e->own_stream;
  return GPDLA_OK;
}

int gpdla_engine_use_null_stream(gpdla_engine* e) {
  if (!e) return set_error(GPDLA_EINVAL, "null engine");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  e->stream = nullptr;  // the null stream (HIP's stream 0)
  return GPDLA_OK;
}

int gpdla_engine_set_panel_streams(gpdla_engine* e, int32_t n) {
  if (!e) return set_error(GPDLA_EINVAL, "null engine");
  if (n < 1 || n > gpdla_engine::kMaxPanelStreams)
    return set_error(GPDLA_EINVAL, "panel streams must be 1..%d (got %d)", gpdla_engine::kMaxPanelStreams, (int)n);
  e->panel_streams = n;
  return GPDLA_OK;
}

// Panel-GEMM path for one batch: per spectrum and chunk of samples, weights -> GEMM on the matrix
// cores (int8 digits, gemm_i8.hip, or fp64, gemm_f64.hip) -> batched LDL^T (gemm_path.hip), in
// stream order.
// A batch's spectra alternate over two streams (gpdla_engine_set_panel_streams), which
// fills the last partial round of each spectrum's weights / LDL^T launches with the other spectrum's
// work: +3.6% on configs[4] (profiles/round5/ab/r11a).  (Earlier second-stream layouts, within one
// spectrum, measured no gain: the LDL^T beside the next chunk's weights and GEMM, 0% with the
// matrix-core LDL^T (profiles/r2f); the weights beside the previous chunk's GEMM, +0.5% (profiles/r2c).)
static int run_panel_gemm(gpdla_engine* e, bool i8, int64_t nq, const int64_t* h_sb, const int64_t* h_lb,
                          const int64_t* h_cap, const int64_t* h_cb, int64_t sc_max, double* o_sll,
                          int64_t ld, double* o_null, hipStream_t st) {
  const int K = e->K;
  const int64_t E = (int64_t)K * (K + 1) / 2;
  const int64_t rows = (sc_max + 127) / 128 * 128;
  // several compute streams: spectrum q on stream q % ns with workspace set q % ns, forked
  // from and joined back into st (the batch's prep / convert before, its reduce after)
  const int ns = (int)std::min<int64_t>(e->panel_streams, nq);
  if (ns > 1) {
    if (!e->panel_fork) HIP_TRY(hipEventCreateWithFlags(&e->panel_fork, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(e->panel_fork, st));
    for (int i = 1; i < ns; ++i) {
      if (!e->panel_stream[i]) HIP_TRY(hipStreamCreateWithFlags(&e->panel_stream[i], hipStreamNonBlocking));
      if (!e->panel_join[i]) HIP_TRY(hipEventCreateWithFlags(&e->panel_join[i], hipEventDisableTiming));
      HIP_TRY(hipStreamWaitEvent(e->panel_stream[i], e->panel_fork, 0));
    }
  }
  const hipStream_t st0 = st;
  auto enqueue = [&]() -> int {
    for (int64_t q = 0; q < nq; ++q) {
      const int set = (int)(q % ns);
      st = set ? e->panel_stream[set] : st0;
      double *G = e->d_G + set * e->ws_G, *U = e->d_U + set * e->ws_U;
      double *q1p = e->d_q1p + set * e->ws_wp, *ldp = e->d_ldp + set * e->ws_wp;
      for (int64_t s0 = 0; s0 <= e->S; s0 += sc_max) {
        const int32_t sc = (int32_t)std::min<int64_t>(sc_max, e->S + 1 - s0);
        if (i8) {  // int8 Ozaki contraction (gemm_i8.hip): weights digits -> exact GEMM -> Gram, u
          const int64_t ks = i8_gemm_kstride(h_cap[q]);
          const int nd = i8_spectrum_nd(e->i8_nd, h_cap[q]);  // short spectra: 32-bit digits (internal.h)
          uint8_t* adig = e->d_ai8 + set * e->ws_ai8;
          WeightsI8Args wi{};
          wi.info = e->d_info; wi.q = (int32_t)q;
          wi.srow = e->d_srow + h_sb[q] * 8; wi.lam_pad = e->d_lam + h_lb[q]; wi.kstride = ks;
          wi.offsets = e->d_off; wi.nhi = e->d_nhi; wi.S = e->S; wi.s0 = s0; wi.sc = sc; wi.rows = rows;
          wi.lines = make_line_args(e->d_lines); wi.nd = nd; wi.adig = adig; wi.q1p = q1p; wi.ldp = ldp;
          HIP_TRY(launch_weights_i8(wi, st));
          GemmI8Args gi{};
          gi.info = e->d_info; gi.q = (int32_t)q; gi.k = K; gi.kstride = ks; gi.rows = rows; gi.sc = sc; gi.nd = nd;
          gi.adig = adig; gi.bdig = e->d_pi8 + h_cb[q];
          gi.ent = e->d_pent + q * 2 * (int64_t)i8_gemm_entries(K); gi.G = G; gi.U = U;
          // the 24-bit path stores the Gram in fp32 (half the GEMM -> LDL^T round trip; adds ~1e-8
          // to its ~2e-7 from fp64, tests/support/emulate_i8.py), in the same workspace
          gi.G32 = nd == 3 ? reinterpret_cast<float*>(G) : nullptr;
          gi.ks_bound = i8_ks_bound(h_cap[q]);  // slot_cap = 4 ceil(lpix / 4) + 16
          TimedLaunch tg{};
          int rc;
          if ((rc = record_start(e, &tg, 3, st))) return rc;
          HIP_TRY(launch_gemm_i8(gi, st));
          HIP_TRY(hipEventRecord(tg.stop, st));
          e->pending.push_back(tg);
        } else {
          WeightsArgs wa{};
          wa.info = e->d_info; wa.q = (int32_t)q;
          wa.srow = e->d_srow + h_sb[q] * 8; wa.lam_pad = e->d_lam + h_lb[q]; wa.cap = h_cap[q];
          wa.offsets = e->d_off; wa.nhi = e->d_nhi; wa.S = e->S; wa.s0 = s0; wa.sc = sc;
          wa.num_lines = e->params.num_lines; wa.lines = make_line_args(e->d_lines);
          double *wg = e->d_wg + set * e->ws_w, *wu = e->d_wu + set * e->ws_w;
          wa.wg = wg; wa.wu = wu; wa.q1p = q1p; wa.ldp = ldp;
          HIP_TRY(launch_weights(wa, st));
          // Gram[s][e] = sum_t Wg[t][s] PG[t][e] (the slot-major Khatri-Rao rows), u[s][i] likewise
          // over the M rows, on the f64 matrix cores (gemm_f64.hip)
          GemmF64Args ga{};
          ga.seg[0] = GemmF64Seg{wg, e->d_panel + h_sb[q] * gemm_ldp(K), gemm_ldp(K), (int32_t)E, G};
          ga.seg[1] = GemmF64Seg{wu, e->d_pm + h_sb[q] * gemm_ldm(K), gemm_ldm(K), K, U};
          ga.nseg = 2;
          ga.cap = h_cap[q]; ga.cap16 = gemm_f64_cap16(h_cap[q]); ga.sc = sc;
          TimedLaunch tg{};
          int rc;
          if ((rc = record_start(e, &tg, 3, st))) return rc;
          HIP_TRY(launch_gemm_f64(ga, st));
          HIP_TRY(hipEventRecord(tg.stop, st));
          e->pending.push_back(tg);
        }
        LdlArgs da{};
        da.info = e->d_info; da.q = (int32_t)q; da.k = K;
        da.G = G; da.U = U; da.q1p = q1p; da.ldp = ldp;
        da.G32 = (i8 && i8_spectrum_nd(e->i8_nd, h_cap[q]) == 3) ? reinterpret_cast<const float*>(G) : nullptr;
        da.S = e->S; da.s0 = s0; da.sc = sc; da.perm = e->d_perm;
        da.sample_ll = o_sll ? o_sll + q * ld : nullptr; da.ll_null = o_null + q; da.status = e->d_status;
        HIP_TRY(launch_ldl_batch(da, st));
      }
    }
    return GPDLA_OK;
  };
  const int rc = enqueue();
  // joined even after a failed enqueue: later work on st0 (the next batch reusing the workspace sets,
  // the engine's synchronize) stays ordered after everything already on the other streams
  for (int i = 1; i < ns; ++i) {
    HIP_TRY(hipEventRecord(e->panel_join[i], e->panel_stream[i]));
    HIP_TRY(hipStreamWaitEvent(st0, e->panel_join[i], 0));
  }
  return rc;
}

// The host-buffer pipeline's stages, sized for the largest batch of this call (no reallocation
// while copies or kernels may still use a stage), its copy stream and events.
static int host_stages_prepare(gpdla_engine* e, int64_t max_pix, int64_t max_q) {
  if (!e->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&e->copy_stream, hipStreamNonBlocking));
  for (HostStage& h : e->hs) {
    int rc;
    if ((rc = grow(&h.wl, &h.cap_wl, (size_t)max_pix))) return rc;
    if ((rc = grow(&h.flux, &h.cap_flux, (size_t)max_pix))) return rc;
    if ((rc = grow(&h.noise, &h.cap_noise, (size_t)max_pix))) return rc;
    if ((rc = grow(&h.mask, &h.cap_mask, (size_t)max_pix))) return rc;
    if ((rc = grow(&h.z, &h.cap_z, (size_t)max_q))) return rc;
    if ((rc = grow(&h.sll, &h.cap_sll, (size_t)(max_q * e->S)))) return rc;
    if ((rc = grow(&h.llnull, &h.cap_o[0], (size_t)max_q))) return rc;
    if ((rc = grow(&h.lldla, &h.cap_o[1], (size_t)max_q))) return rc;
    if ((rc = grow(&h.zmin, &h.cap_o[2], (size_t)max_q))) return rc;
    if ((rc = grow(&h.zmax, &h.cap_o[3], (size_t)max_q))) return rc;
    if ((rc = grow(&h.npix, &h.cap_o[4], (size_t)max_q))) return rc;
    for (hipEvent_t* ev : {&h.in_ready, &h.in_free, &h.out_ready, &h.out_free})
      if (!*ev) HIP_TRY(hipEventCreateWithFlags(ev, hipEventDisableTiming));
  }
  return GPDLA_OK;
}

// Batch [q0, q0 + nq)'s results from its stage back to the host, on the copy stream once the
// compute stream has written them.  With pageable host memory the call returns when the copy is
// done; the caller has already queued the next batch's kernels, so the device keeps computing.
static int host_stage_copy_out(gpdla_engine* e, const gpdla_results* res, int64_t bi, int64_t q0, int64_t nq) {
  HostStage& h = e->hs[bi & 1];
  hipStream_t cs = e->copy_stream;
  HIP_TRY(hipStreamWaitEvent(cs, h.out_ready, 0));
  HIP_TRY(hipMemcpyAsync(res->log_likelihoods_no_dla + q0, h.llnull, nq * 8, hipMemcpyDeviceToHost, cs));
  HIP_TRY(hipMemcpyAsync(res->log_likelihoods_dla + q0, h.lldla, nq * 8, hipMemcpyDeviceToHost, cs));
  if (res->min_z_dlas) HIP_TRY(hipMemcpyAsync(res->min_z_dlas + q0, h.zmin, nq * 8, hipMemcpyDeviceToHost, cs));
  if (res->max_z_dlas) HIP_TRY(hipMemcpyAsync(res->max_z_dlas + q0, h.zmax, nq * 8, hipMemcpyDeviceToHost, cs));
  if (res->num_pixels) HIP_TRY(hipMemcpyAsync(res->num_pixels + q0, h.npix, nq * 4, hipMemcpyDeviceToHost, cs));
  if (res->sample_log_likelihoods_dla)
    HIP_TRY(hipMemcpy2DAsync(res->sample_log_likelihoods_dla + q0 * res->sample_ld, res->sample_ld * 8, h.sll,
                             e->S * 8, e->S * 8, nq, hipMemcpyDeviceToHost, cs));
  HIP_TRY(hipEventRecord(h.out_free, cs));
  return GPDLA_OK;
}

int gpdla_engine_process(gpdla_engine* e, const gpdla_spectra* sp, const gpdla_results* res) {
  if (!e || !sp || !res) return set_error(GPDLA_EINVAL, "null argument");
  const int64_t Q = sp->num_spectra;
  if (Q < 0) return set_error(GPDLA_EINVAL, "num_spectra < 0");
  if (Q == 0) return GPDLA_OK;
  if (!sp->offsets || !sp->wavelengths || !sp->flux || !sp->noise_variance || !sp->pixel_mask || !sp->z_qsos)
    return set_error(GPDLA_EINVAL, "null spectra array");
  if (!res->log_likelihoods_no_dla || !res->log_likelihoods_dla)
    return set_error(GPDLA_EINVAL, "null result array");
  if (res->sample_log_likelihoods_dla && res->sample_ld < e->S)
    return set_error(GPDLA_EINVAL, "sample_ld (%lld) < num_samples (%lld)", (long long)res->sample_ld,
                     (long long)e->S);
  if (sp->offsets[0] < 0) return set_error(GPDLA_EINVAL, "offsets[0] < 0");
  for (int64_t q = 0; q < Q; ++q)
    if (sp->offsets[q + 1] < sp->offsets[q]) return set_error(GPDLA_EINVAL, "offsets not monotone at %lld", (long long)q);
  const bool in_dev = sp->memory == GPDLA_MEM_DEVICE, out_dev = res->memory == GPDLA_MEM_DEVICE;
  HIP_TRY(hipSetDevice(e->device));
  hipStream_t st = e->stream;

  const int64_t QB = e->params.max_batch_spectra > 0 ? e->params.max_batch_spectra : (e->gemm ? 64 : 1024);
  // panel doubles per slot: fused layout row, or the Khatri-Rao row of the panel-GEMM layout
  const int64_t E = (int64_t)e->K * (e->K + 1) / 2;
  const int64_t row = e->gemm ? gemm_ldp(e->K) : panel_row_doubles(e->K);
  const int es = e->gemm ? 0 : scratch_doubles(e->K);
  // panel-GEMM sample chunks: the S + 1 samples (null model included) in equal chunks of at most
  // kMaxChunk.  configs[4] (S + 1 = 100,001) measured 46.2 Mevals/s with 16,384-sample chunks (6
  // full + a 1,697-sample tail that fills a sixth of the GPU), 47.4 with 7 equal chunks, 48.5 with
  // 2 and 49.1 with one (profiles/r2l); again after the round-2 GEMM work: 53.5 (6 equal chunks),
  // 58.8 (4), 61.7 (2), 63.1 (one; profiles/r2/c5_ab): smaller chunks keep the A digits in the
  // Infinity Cache (GEMM -10%) but cost more in the weights and LDL^T launches.  The chunk is also
  // capped per batch by a workspace budget (panel_chunk below): per sample, the A digits (8 B per
  // slot) or the fp64 weights (16 B per slot), plus the Gram and u (8 (k(k+1)/2 + k) B).
  constexpr int64_t kMaxChunk = GPDLA_MAX_CHUNK;
  const int64_t blocks_x = (e->S + 1 + kSamplesPerBlock - 1) / kSamplesPerBlock;

  // pinned metadata for every batch of this call: per batch (QB+1) + 4*QB int64
  const size_t per_batch = (size_t)(QB + 1) + 4 * (size_t)QB;
  const int64_t nbatch = (Q + QB - 1) / QB;
  HIP_TRY(hipEventSynchronize(e->meta_done));
  if (e->cap_hmeta < per_batch * nbatch) {
    if (e->h_meta) (void)hipHostFree(e->h_meta);
    e->h_meta = nullptr;
    e->cap_hmeta = 0;
    HIP_TRY(hipHostMalloc((void**)&e->h_meta, per_batch * nbatch * sizeof(int64_t)));
    e->cap_hmeta = per_batch * nbatch;
  }

  // host inputs and host results: the two-stage pipeline (copies beside the kernels)
  const bool pipe = !in_dev && !out_dev;
  if (pipe) {
    int64_t max_pix = 0;
    for (int64_t bi = 0; bi < nbatch; ++bi)
      max_pix = std::max(max_pix, sp->offsets[std::min(Q, (bi + 1) * QB)] - sp->offsets[bi * QB]);
    int rc;
    // no copy or kernel of an earlier call (one that returned an error mid-loop included) may still
    // use a stage that host_stages_prepare is about to free and grow
    if (e->copy_stream) HIP_TRY(hipStreamSynchronize(e->copy_stream));
    HIP_TRY(hipStreamSynchronize(st));
    if ((rc = host_stages_prepare(e, max_pix, std::min(Q, QB)))) return rc;
    // order this call after any other work on the engine's stream, then keep the two streams apart
    // except through the events
    HIP_TRY(hipStreamSynchronize(e->copy_stream));
    for (HostStage& h : e->hs) {
      HIP_TRY(hipEventRecord(h.in_free, st));
      HIP_TRY(hipEventRecord(h.out_free, e->copy_stream));
    }
  }

  for (int64_t bi = 0; bi < nbatch; ++bi) {
    const int64_t q0 = bi * QB, q1 = std::min(Q, q0 + QB), nq = q1 - q0;
    HostStage& hst = e->hs[bi & 1];
    int64_t* hm = e->h_meta + bi * per_batch;
    int64_t* h_off = hm;
    int64_t* h_sb = hm + (QB + 1);
    int64_t* h_lb = h_sb + QB;
    int64_t* h_cap = h_lb + QB;
    int64_t* h_cb = h_cap + QB;  // int8 path: first chunk of each spectrum
    int64_t slots = 0, lams = 0, cap_max = 0, chunks = 0, lpix_max = 0;
    for (int64_t q = 0; q < nq; ++q) {
      h_off[q] = sp->offsets[q0 + q] - sp->offsets[q0];
      const int64_t lpix = sp->offsets[q0 + q + 1] - sp->offsets[q0 + q];
      const int64_t cap = 4 * ((lpix + 3) / 4) + 4 * kChunkSteps;
      h_sb[q] = slots;
      h_lb[q] = lams;
      h_cap[q] = cap;
      if (e->gemm) {  // int8 panel-GEMM: byte base of the spectrum's B digit planes
        h_cb[q] = chunks;
        chunks += 4 * (int64_t)i8_gemm_entries(e->K) * i8_gemm_kstride(cap);
      } else {
        h_cb[q] = chunks;
        chunks += ((lpix + 3) / 4 + 15) / 16;  // >= ceil(L / 16) chunks of 16 steps per segment
      }
      lpix_max = std::max(lpix_max, lpix);
      cap_max = std::max(cap_max, cap);
      slots += cap;
      lams += cap + 8;
    }
    h_off[nq] = sp->offsets[q1] - sp->offsets[q0];
    const int64_t npix = h_off[nq];
    // int8 contraction for this batch: its int32 level sums are exact only up to kI8MaxSlots
    // slots, so a batch holding a longer spectrum runs the fp64 kernels (fused or dgemm) instead
    const bool i8_exact = lpix_max <= kI8MaxSlots;
    const bool batch_i8 = e->i8 && !e->gemm && i8_exact;
    const bool batch_gemm_i8 = e->i8 && e->gemm && i8_exact;
    // panel-GEMM sample chunk of this batch: equal chunks of at most kMaxChunk samples whose
    // workspaces fit the budget (a quarter of the free device memory, at most 16 GiB)
    int64_t sc_max = 0;
    if (e->gemm) {
      size_t free_b = 0, total_b = 0;
      HIP_TRY(hipMemGetInfo(&free_b, &total_b));
      const int64_t budget = (int64_t)std::min<size_t>(free_b / 4, (size_t)16 << 30);
      // (one workspace set per panel stream)
      const int64_t per_sample = e->panel_streams *
                                 ((batch_gemm_i8 ? 8 * i8_gemm_kstride(cap_max) : 16 * gemm_f64_cap16(cap_max)) +
                                  8 * (E + e->K + 2 * kWeightParts));
      const int64_t fit = std::max<int64_t>(128, budget / std::max<int64_t>(per_sample, 1) / 128 * 128);
      const int64_t cmax = std::min<int64_t>(kMaxChunk, fit);
      const int64_t nchunk = (e->S + 1 + cmax - 1) / cmax;
      sc_max = (e->S + 1 + nchunk - 1) / nchunk;
    }

    int rc;
    if ((rc = grow(&e->d_meta, &e->cap_meta, per_batch))) return rc;
    if ((rc = grow(&e->d_info, &e->cap_q, (size_t)QB))) return rc;
    // + one LDS row of slack: the staging DMA reads whole 1 KiB pieces (kernels.hip stage_chunk).  The
    // int8 panel batches never read the Khatri-Rao panel (prep skips it, convert_gemm_i8_kernel forms
    // the products from the M rows), so they do not grow it (a few hundred MB at k = 50)
    if (!batch_gemm_i8 &&
        (rc = grow(&e->d_panel, &e->cap_slots,
                   (size_t)(slots * row + (e->gemm ? gemm_panel_slack(row) : panel_lds_row_doubles(e->K)))))) return rc;
    if ((rc = grow(&e->d_lam, &e->cap_lam, (size_t)lams))) return rc;
    if (e->gemm) {
      const int64_t ldm = gemm_ldm(e->K);
      if ((rc = grow(&e->d_pm, &e->cap_pm, (size_t)(slots * ldm + gemm_panel_slack(ldm))))) return rc;
      // the rows gemm_f64 reads past the batch's last slot: zero (finite, against zero weights)
      if (!batch_gemm_i8) HIP_TRY(hipMemsetAsync(e->d_panel + slots * row, 0, gemm_panel_slack(row) * 8, st));
      HIP_TRY(hipMemsetAsync(e->d_pm + slots * ldm, 0, gemm_panel_slack(ldm) * 8, st));
      if ((rc = grow(&e->d_srow, &e->cap_srow, (size_t)slots * 8))) return rc;
      const int64_t sets = e->panel_streams;  // one workspace set per panel stream
      if (!batch_gemm_i8) {  // the fp64 weight tiles: only the fp64 GEMM reads them
        e->ws_w = gemm_f64_cap16(cap_max) * gemm_f64_rows(sc_max);
        if ((rc = grow(&e->d_wg, &e->cap_wg, (size_t)(sets * e->ws_w)))) return rc;
        if ((rc = grow(&e->d_wu, &e->cap_wu, (size_t)(sets * e->ws_w)))) return rc;
      }
      // the GEMMs store whole 128-sample tiles (quad_index layout, internal.h); + 64 elements of
      // slack: ldl_mfma_kernel's straight-line tile loads may address one entry past the last
      // sample's Gram when k is a multiple of 4 (the value is discarded)
      const int64_t grows = gemm_f64_rows(sc_max);
      e->ws_G = E * grows + 64;
      e->ws_U = e->K * grows + 64;
      e->ws_wp = kWeightParts * sc_max;
      if ((rc = grow(&e->d_G, &e->cap_G, (size_t)(sets * e->ws_G)))) return rc;
      if ((rc = grow(&e->d_U, &e->cap_U, (size_t)(sets * e->ws_U)))) return rc;
      if ((rc = grow(&e->d_q1p, &e->cap_q1p, (size_t)(sets * e->ws_wp)))) return rc;
      if ((rc = grow(&e->d_ldp, &e->cap_ldp, (size_t)(sets * e->ws_wp)))) return rc;
    }
    if (batch_gemm_i8) {
      if ((rc = grow(&e->d_pi8, &e->cap_pi8, (size_t)chunks))) return rc;
      if ((rc = grow(&e->d_pent, &e->cap_pent, (size_t)nq * 2 * i8_gemm_entries(e->K)))) return rc;
      e->ws_ai8 = (int64_t)8 * ((sc_max + 127) / 128 * 128) * i8_gemm_kstride(cap_max + 0);
      if ((rc = grow(&e->d_ai8, &e->cap_ai8, (size_t)(e->panel_streams * e->ws_ai8)))) return rc;
    }
    if (batch_i8) {  // (the fp64 fused kernel transposes its accumulators in registers: no scratch)
      if ((rc = grow(&e->d_scratch, &e->cap_scr, (size_t)blocks_x * nq * kSamplesPerBlock * es))) return rc;
      if ((rc = grow(&e->d_pi8, &e->cap_pi8, (size_t)chunks * i8_chunk_bytes(e->K)))) return rc;
      if ((rc = grow(&e->d_psc, &e->cap_psc, (size_t)chunks * 64 * 8))) return rc;
      if ((rc = grow(&e->d_pent, &e->cap_pent, (size_t)nq * 2 * i8_entries(e->K)))) return rc;
    }
    if ((rc = grow(&e->d_smap, &e->cap_smap, (size_t)slots))) return rc;
    HIP_TRY(hipMemcpyAsync(e->d_meta, hm, per_batch * sizeof(int64_t), hipMemcpyHostToDevice, st));

    const double *wl, *fl, *nv, *zq;
    const uint8_t* mk;
    const int64_t pbase = sp->offsets[q0];
    if (in_dev) {
      wl = sp->wavelengths + pbase; fl = sp->flux + pbase; nv = sp->noise_variance + pbase;
      mk = sp->pixel_mask + pbase; zq = sp->z_qsos + q0;
    } else if (pipe) {
      // into this batch's stage once batch bi - 2's prep_kernel has read it, beside batch bi - 1
      hipStream_t cs = e->copy_stream;
      HIP_TRY(hipStreamWaitEvent(cs, hst.in_free, 0));
      HIP_TRY(hipMemcpyAsync(hst.wl, sp->wavelengths + pbase, npix * 8, hipMemcpyHostToDevice, cs));
      HIP_TRY(hipMemcpyAsync(hst.flux, sp->flux + pbase, npix * 8, hipMemcpyHostToDevice, cs));
      HIP_TRY(hipMemcpyAsync(hst.noise, sp->noise_variance + pbase, npix * 8, hipMemcpyHostToDevice, cs));
      HIP_TRY(hipMemcpyAsync(hst.mask, sp->pixel_mask + pbase, npix, hipMemcpyHostToDevice, cs));
      HIP_TRY(hipMemcpyAsync(hst.z, sp->z_qsos + q0, nq * 8, hipMemcpyHostToDevice, cs));
      HIP_TRY(hipEventRecord(hst.in_ready, cs));
      HIP_TRY(hipStreamWaitEvent(st, hst.in_ready, 0));
      wl = hst.wl; fl = hst.flux; nv = hst.noise; mk = hst.mask; zq = hst.z;
    } else {
      if ((rc = grow(&e->d_wl, &e->cap_wl, (size_t)npix))) return rc;
      if ((rc = grow(&e->d_flux, &e->cap_flux, (size_t)npix))) return rc;
      if ((rc = grow(&e->d_noise, &e->cap_noise, (size_t)npix))) return rc;
      if ((rc = grow(&e->d_mask, &e->cap_mask, (size_t)npix))) return rc;
      if ((rc = grow(&e->d_z, &e->cap_z, (size_t)nq))) return rc;
      HIP_TRY(hipMemcpyAsync(e->d_wl, sp->wavelengths + pbase, npix * 8, hipMemcpyHostToDevice, st));
      HIP_TRY(hipMemcpyAsync(e->d_flux, sp->flux + pbase, npix * 8, hipMemcpyHostToDevice, st));
      HIP_TRY(hipMemcpyAsync(e->d_noise, sp->noise_variance + pbase, npix * 8, hipMemcpyHostToDevice, st));
      HIP_TRY(hipMemcpyAsync(e->d_mask, sp->pixel_mask + pbase, npix, hipMemcpyHostToDevice, st));
      HIP_TRY(hipMemcpyAsync(e->d_z, sp->z_qsos + q0, nq * 8, hipMemcpyHostToDevice, st));
      wl = e->d_wl; fl = e->d_flux; nv = e->d_noise; mk = e->d_mask; zq = e->d_z;
    }

    // outputs: device results are written in place; host results go through workspaces
    double *o_sll, *o_null, *o_dla, *o_zmin, *o_zmax;
    int32_t* o_npix;
    int64_t ld;
    const bool need_internal_sll = !pipe && (!out_dev || !res->sample_log_likelihoods_dla);
    if (need_internal_sll) {
      if ((rc = grow(&e->d_sll, &e->cap_sll, (size_t)nq * e->S))) return rc;
    }
    if (out_dev) {
      o_sll = res->sample_log_likelihoods_dla ? res->sample_log_likelihoods_dla + q0 * res->sample_ld : e->d_sll;
      ld = res->sample_log_likelihoods_dla ? res->sample_ld : e->S;
      o_null = res->log_likelihoods_no_dla + q0;
      o_dla = res->log_likelihoods_dla + q0;
      o_zmin = res->min_z_dlas ? res->min_z_dlas + q0 : nullptr;
      o_zmax = res->max_z_dlas ? res->max_z_dlas + q0 : nullptr;
      o_npix = res->num_pixels ? res->num_pixels + q0 : nullptr;
    } else if (pipe) {
      // this batch's stage, once batch bi - 2's results have left it
      HIP_TRY(hipStreamWaitEvent(st, hst.out_free, 0));
      o_sll = hst.sll; ld = e->S;
      o_null = hst.llnull; o_dla = hst.lldla; o_zmin = hst.zmin; o_zmax = hst.zmax; o_npix = hst.npix;
    } else {
      if (e->cap_qout < (size_t)QB) {
        for (double** p : {&e->d_llnull, &e->d_lldla, &e->d_zmin, &e->d_zmax})
          if (*p) { (void)hipFree(*p); *p = nullptr; }
        if (e->d_npix) { (void)hipFree(e->d_npix); e->d_npix = nullptr; }
        size_t a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0;
        if ((rc = grow(&e->d_llnull, &a1, (size_t)QB))) return rc;
        if ((rc = grow(&e->d_lldla, &a2, (size_t)QB))) return rc;
        if ((rc = grow(&e->d_zmin, &a3, (size_t)QB))) return rc;
        if ((rc = grow(&e->d_zmax, &a4, (size_t)QB))) return rc;
        if ((rc = grow(&e->d_npix, &a5, (size_t)QB))) return rc;
        e->cap_qout = QB;
      }
      o_sll = e->d_sll; ld = e->S;
      o_null = e->d_llnull; o_dla = e->d_lldla; o_zmin = e->d_zmin; o_zmax = e->d_zmax; o_npix = e->d_npix;
    }

    PrepArgs pa{};
    pa.q_count = (int32_t)nq;
    pa.offsets = e->d_meta;
    pa.wavelengths = wl; pa.flux = fl; pa.noise = nv; pa.mask = mk; pa.z_qsos = zq;
    pa.slot_base = e->d_meta + (QB + 1);
    pa.lam_base = pa.slot_base + QB;
    pa.slot_cap = pa.lam_base + QB;
    pa.num_rest = e->num_rest;
    pa.rest = e->d_rest; pa.mu = e->d_mu; pa.M_rowmajor = e->d_M; pa.log_omega = e->d_logom;
    pa.c_0 = e->c0; pa.tau_0 = e->tau0; pa.beta = e->beta;
    pa.min_lambda = e->params.min_lambda; pa.max_lambda = e->params.max_lambda;
    pa.lya = e->params.lya_wavelength; pa.lyman_limit = e->params.lyman_limit;
    pa.min_z_cut = e->params.min_z_cut; pa.max_z_cut = e->params.max_z_cut;
    pa.pixel_spacing = e->params.pixel_spacing;
    pa.absorption_mode = e->params.absorption_mode;
    pa.om2_hi_e = e->om2_hi_e;
    pa.info = e->d_info; pa.panel = e->d_panel; pa.lam_pad = e->d_lam; pa.slot_pixel = e->d_smap;
    pa.k = e->K; pa.panel_m = e->d_pm; pa.srow = e->d_srow;
    // the int8 panel paths form the Khatri-Rao entries from the M rows (convert_gemm_i8_kernel): prep
    // skips the k(k+1)/2 doubles per slot
    if (batch_gemm_i8) pa.panel = nullptr;

    LikelihoodArgs la{};
    la.q_count = (int32_t)nq;
    la.info = e->d_info; la.panel = e->d_panel; la.lam_pad = e->d_lam;
    la.offsets = e->d_off; la.nhi = e->d_nhi; la.perm = e->d_perm; la.S = e->S;
    la.num_lines = e->params.num_lines;
    la.lines = make_line_args(e->d_lines);
    la.sample_ll = o_sll; la.ld = ld; la.ll_null = o_null; la.status = e->d_status;

    ConvertI8Args ca{};
    LikelihoodI8Args li{};
    if (batch_i8) {
      ca.q_count = (int32_t)nq; ca.info = e->d_info; ca.panel = e->d_panel; ca.lam_pad = e->d_lam;
      ca.chunk_base = pa.slot_cap + QB; ca.panel_i8 = e->d_pi8; ca.scal = e->d_psc; ca.ent = e->d_pent;
      li.q_count = (int32_t)nq; li.info = e->d_info; li.panel_i8 = e->d_pi8; li.scal = e->d_psc;
      li.ent = e->d_pent; li.chunk_base = ca.chunk_base; li.lam_pad = e->d_lam;
      li.offsets = e->d_off; li.nhi = e->d_nhi; li.perm = e->d_perm; li.S = e->S;
      li.lines = la.lines; li.scratch = e->d_scratch;
      li.sample_ll = o_sll; li.ld = ld; li.ll_null = o_null; li.status = e->d_status;
    }

    ReduceArgs ra{};
    ra.q_count = (int32_t)nq; ra.info = e->d_info; ra.sample_ll = o_sll; ra.ld = ld; ra.S = e->S;
    ra.ll_dla = o_dla; ra.zmin = o_zmin; ra.zmax = o_zmax; ra.num_pixels = o_npix;

    TimedLaunch t0{}, t1{}, t2{};
    if ((rc = record_start(e, &t0, 0))) return rc;
    HIP_TRY(launch_prep(e->gemm ? 0 : e->K, pa, st));
    if (pipe) HIP_TRY(hipEventRecord(hst.in_free, st));
    if (batch_i8) HIP_TRY(launch_convert_i8(e->K, ca, st));
    if (batch_gemm_i8) {
      ConvertGemmI8Args cg{};
      cg.k = e->K; cg.info = e->d_info; cg.panel_m = e->d_pm; cg.srow = e->d_srow;
      cg.slot_base = pa.slot_base; cg.slot_cap = pa.slot_cap; cg.bbase = pa.slot_cap + QB;
      cg.bdig = e->d_pi8; cg.ent = e->d_pent; cg.nd = e->i8_nd;
      HIP_TRY(launch_convert_gemm_i8(cg, (int32_t)nq, st));
    }
    HIP_TRY(hipEventRecord(t0.stop, st));
    e->pending.push_back(t0);
    if ((rc = record_start(e, &t1, 1))) return rc;
    if (batch_i8) {
      HIP_TRY(launch_likelihood_i8(e->K, li, st));
    } else if (!e->gemm) {
      HIP_TRY(launch_likelihood(e->K, la, st));
    } else if ((rc = run_panel_gemm(e, batch_gemm_i8, nq, h_sb, h_lb, h_cap, h_cb, sc_max, o_sll, ld, o_null, st))) {
      return rc;
    }
    HIP_TRY(hipEventRecord(t1.stop, st));
    e->pending.push_back(t1);

    if ((rc = record_start(e, &t2, 2))) return rc;
    HIP_TRY(launch_reduce(ra, st));
    HIP_TRY(hipEventRecord(t2.stop, st));
    e->pending.push_back(t2);

    e->stats.spectra += nq;
    e->stats.sample_evals += nq * e->S;

    if (pipe) {
      HIP_TRY(hipEventRecord(hst.out_ready, st));
      // the previous batch's results, now that this batch is queued behind it
      if (bi > 0 && (rc = host_stage_copy_out(e, res, bi - 1, q0 - QB, QB))) return rc;
    } else if (!out_dev) {
      HIP_TRY(hipMemcpyAsync(res->log_likelihoods_no_dla + q0, o_null, nq * 8, hipMemcpyDeviceToHost, st));
      HIP_TRY(hipMemcpyAsync(res->log_likelihoods_dla + q0, o_dla, nq * 8, hipMemcpyDeviceToHost, st));
      if (res->min_z_dlas) HIP_TRY(hipMemcpyAsync(res->min_z_dlas + q0, o_zmin, nq * 8, hipMemcpyDeviceToHost, st));
      if (res->max_z_dlas) HIP_TRY(hipMemcpyAsync(res->max_z_dlas + q0, o_zmax, nq * 8, hipMemcpyDeviceToHost, st));
      if (res->num_pixels) HIP_TRY(hipMemcpyAsync(res->num_pixels + q0, o_npix, nq * 4, hipMemcpyDeviceToHost, st));
      if (res->sample_log_likelihoods_dla)
        HIP_TRY(hipMemcpy2DAsync(res->sample_log_likelihoods_dla + q0 * res->sample_ld, res->sample_ld * 8,
                                 o_sll, e->S * 8, e->S * 8, nq, hipMemcpyDeviceToHost, st));
      // host results: the workspaces are reused by the next batch, so drain here
      HIP_TRY(hipStreamSynchronize(st));
    } else if (!in_dev) {
      // host inputs were staged in reusable workspaces
      HIP_TRY(hipStreamSynchronize(st));
    }
    // otherwise the next batch reuses the panel workspace in stream order
  }
  if (pipe) {
    const int64_t bl = nbatch - 1;
    const int rc = host_stage_copy_out(e, res, bl, bl * QB, Q - bl * QB);
    if (rc) return rc;
  }
  HIP_TRY(hipEventRecord(e->meta_done, st));
  if (pipe) HIP_TRY(hipStreamSynchronize(e->copy_stream));
  if (!out_dev) return gpdla_engine_synchronize(e);
  return GPDLA_OK;
}

int gpdla_engine_synchronize(gpdla_engine* e) {
  if (!e) return set_error(GPDLA_EINVAL, "null engine");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  int rc = resolve_events(e);
  if (rc) return rc;
  int32_t status = 0;
  HIP_TRY(hipMemcpy(&status, e->d_status, 4, hipMemcpyDeviceToHost));
  if (status) {
    HIP_TRY(hipMemset(e->d_status, 0, 4));
    return set_error(GPDLA_ENUMERIC, "non-positive pivot or non-finite likelihood (outputs NaN)");
  }
  return GPDLA_OK;
}

int gpdla_engine_get_stats_n(gpdla_engine* e, gpdla_stats* s, int64_t stats_bytes) {
  if (!e || !s || stats_bytes < 0) return set_error(GPDLA_EINVAL, "null argument");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  int rc = resolve_events(e);
  if (rc) return rc;
  std::memcpy(s, &e->stats, std::min<size_t>((size_t)stats_bytes, sizeof(gpdla_stats)));
  return GPDLA_OK;
}

int gpdla_engine_get_stats(gpdla_engine* e, gpdla_stats* s) {
  return gpdla_engine_get_stats_n(e, s, (int64_t)sizeof(gpdla_stats));
}

int gpdla_engine_reset_stats(gpdla_engine* e) {
  if (!e) return set_error(GPDLA_EINVAL, "null engine");
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipStreamSynchronize(e->stream));
  int rc = resolve_events(e);
  if (rc) return rc;
  e->stats = gpdla_stats{};
  return GPDLA_OK;
}

// ---------------------------------------------------------------------------------------------
// device buffer helpers
// ---------------------------------------------------------------------------------------------
int gpdla_device_malloc(int32_t device, int64_t bytes, void** ptr) {
  if (!ptr || bytes < 0) return set_error(GPDLA_EINVAL, "bad argument");
  *ptr = nullptr;
  int rc = check_device(device);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipMalloc(ptr, bytes > 0 ? bytes : 1));
  return GPDLA_OK;
}

int gpdla_device_free(int32_t device, void* ptr) {
  int rc = check_device(device);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(device));
  if (ptr) HIP_TRY(hipFree(ptr));
  return GPDLA_OK;
}

int gpdla_memcpy_htod(int32_t device, void* dst, const void* src, int64_t bytes) {
  int rc = check_device(device);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return GPDLA_OK;
}

int gpdla_memcpy_dtoh(int32_t device, void* dst, const void* src, int64_t bytes) {
  int rc = check_device(device);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return GPDLA_OK;
}

// ---------------------------------------------------------------------------------------------
// standalone entry points (host buffers)
// ---------------------------------------------------------------------------------------------
static int lines_on_device(double** d_lines) {
  static std::mutex mu;
  static std::vector<double*> per_dev;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(mu);
  if ((int)per_dev.size() <= dev) per_dev.resize(dev + 1, nullptr);
  if (!per_dev[dev]) {
    const std::vector<double>& lines = host_line_data().buf;
    double* p = nullptr;
    HIP_TRY(hipMalloc((void**)&p, lines.size() * 8));
    HIP_TRY(hipMemcpy(p, lines.data(), lines.size() * 8, hipMemcpyHostToDevice));
    per_dev[dev] = p;
  }
  *d_lines = per_dev[dev];
  return GPDLA_OK;
}

// Device and pinned host buffers of the standalone entry points, cached per device and grown on
// demand, plus a non-blocking stream: the MEX drop-ins are called once per
// sample from a MATLAB loop, so a call is one memcpy into pinned memory, one H2D copy, the kernel,
// one D2H copy and a stream synchronisation -- no allocation, no pageable copies, no memset.
// Calls are serialised per device.
struct StandaloneBufs {
  std::mutex mu;
  char* buf = nullptr;    // device
  char* host = nullptr;   // pinned host staging
  size_t cap = 0, hcap = 0;
  hipStream_t stream = nullptr;
};

static StandaloneBufs& standalone_bufs(int dev) {
  static std::mutex mu;
  static std::vector<StandaloneBufs*> per_dev;
  std::lock_guard<std::mutex> lock(mu);
  if ((int)per_dev.size() <= dev) per_dev.resize(dev + 1, nullptr);
  if (!per_dev[dev]) per_dev[dev] = new StandaloneBufs();
  return *per_dev[dev];
}

static hipError_t standalone_reserve(StandaloneBufs& b, size_t bytes, size_t host_bytes) {
  hipError_t e = hipSuccess;
  if (!b.stream) e = hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking);
  if (e == hipSuccess && (bytes > b.cap || !b.buf)) {
    if (b.buf) (void)hipFree(b.buf);
    b.buf = nullptr;
    b.cap = 0;
    e = hipMalloc((void**)&b.buf, bytes);
    if (e == hipSuccess) b.cap = bytes;
  }
  if (e == hipSuccess && (host_bytes > b.hcap || !b.host)) {
    if (b.host) (void)hipHostFree(b.host);
    b.host = nullptr;
    b.hcap = 0;
    e = hipHostMalloc((void**)&b.host, host_bytes);
    if (e == hipSuccess) b.hcap = host_bytes;
  }
  return e;
}

int gpdla_voigt_batch_f64(const double* lambdas, int64_t n_padded, const double* z, const double* N,
                          int64_t count, int32_t num_lines, double* out) {
  if (!lambdas || !z || !N || !out) return set_error(GPDLA_EINVAL, "null argument");
  if (n_padded <= 2 * kWidth) return set_error(GPDLA_EINVAL, "need more than %d wavelengths", 2 * kWidth);
  if (num_lines < 1 || num_lines > kMaxLines) return set_error(GPDLA_EINVAL, "num_lines=%d outside [1, 31]", num_lines);
  if (count < 1) return GPDLA_OK;
  int rc = check_device(0);
  if (rc) return rc;
  double* d_lines = nullptr;
  if ((rc = lines_on_device(&d_lines))) return rc;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  StandaloneBufs& sb = standalone_bufs(dev);
  std::lock_guard<std::mutex> lock(sb.mu);
  const int64_t n_out = n_padded - 2 * kWidth;
  const size_t n_in = (size_t)(n_padded + 2 * count);          // [lambdas | z | N]
  const size_t bytes = (n_in + (size_t)count * n_out) * 8;
  hipError_t err = standalone_reserve(sb, bytes, n_in * 8);
  if (err != hipSuccess) return set_error(GPDLA_EDEVICE, "voigt: %s", hipGetErrorString(err));
  double* h = (double*)sb.host;
  std::memcpy(h, lambdas, n_padded * 8);
  std::memcpy(h + n_padded, z, count * 8);
  std::memcpy(h + n_padded + count, N, count * 8);
  double* d_lam = (double*)sb.buf;
  double* d_z = d_lam + n_padded;
  double* d_N = d_z + count;
  double* d_out = d_N + count;
  err = hipMemcpyAsync(d_lam, h, n_in * 8, hipMemcpyHostToDevice, sb.stream);
  if (err == hipSuccess) err = launch_voigt_batch(d_lam, n_padded, d_z, d_N, count, num_lines, make_line_args(d_lines), d_out, sb.stream);
  // the profiles straight into the caller's buffer (the pinned staging is write-combined: reading
  // it back on the host is slow)
  if (err == hipSuccess) err = hipMemcpyAsync(out, d_out, count * n_out * 8, hipMemcpyDeviceToHost, sb.stream);
  if (err == hipSuccess) err = hipStreamSynchronize(sb.stream);
  if (err != hipSuccess) return set_error(GPDLA_EDEVICE, "voigt: %s", hipGetErrorString(err));
  return GPDLA_OK;
}

int gpdla_diag_raw_profile3(const double* lambdas, int64_t n, double z, double N, int32_t f32, double* out) {
  if (!lambdas || !out) return set_error(GPDLA_EINVAL, "null argument");
  if (n < 1) return GPDLA_OK;
  int rc = check_device(0);
  if (rc) return rc;
  double* d_lines = nullptr;
  if ((rc = lines_on_device(&d_lines))) return rc;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  StandaloneBufs& sb = standalone_bufs(dev);
  std::lock_guard<std::mutex> lock(sb.mu);
  hipError_t err = standalone_reserve(sb, (size_t)n * 16, (size_t)n * 8);
  if (err != hipSuccess) return set_error(GPDLA_EDEVICE, "raw profile: %s", hipGetErrorString(err));
  double* d_lam = (double*)sb.buf;
  double* d_out = d_lam + n;
  std::memcpy(sb.host, lambdas, (size_t)n * 8);
  err = hipMemcpyAsync(d_lam, sb.host, (size_t)n * 8, hipMemcpyHostToDevice, sb.stream);
  if (err == hipSuccess) err = launch_diag_raw_profile(d_lam, n, z, N, f32 ? 1 : 0, make_line_args(d_lines), d_out, sb.stream);
  if (err == hipSuccess) err = hipMemcpyAsync(out, d_out, (size_t)n * 8, hipMemcpyDeviceToHost, sb.stream);
  if (err == hipSuccess) err = hipStreamSynchronize(sb.stream);
  if (err != hipSuccess) return set_error(GPDLA_EDEVICE, "raw profile: %s", hipGetErrorString(err));
  return GPDLA_OK;
}

int gpdla_voigt_f64(const double* lambdas, int64_t n_padded, double z, double N, int32_t num_lines,
                    double* out) {
  return gpdla_voigt_batch_f64(lambdas, n_padded, &z, &N, 1, num_lines, out);
}

int gpdla_log_mvnpdf_low_rank_f64(const double* y, const double* mu, const double* M, const double* d,
                                  int64_t n, int32_t k, double* out) {
  if (!y || !mu || !M || !d || !out) return set_error(GPDLA_EINVAL, "null argument");
  if (n < 1 || k < 1) return set_error(GPDLA_EINVAL, "n=%lld k=%d", (long long)n, k);
  if (k > 64) return set_error(GPDLA_EUNSUPPORTED, "k=%d > 64 in the standalone entry point", k);
  int rc = check_device(0);
  if (rc) return rc;
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  StandaloneBufs& sb = standalone_bufs(dev);
  std::lock_guard<std::mutex> lock(sb.mu);
  // one staging copy: [y | mu | d | M | out | status]
  const size_t nin = (size_t)n * (3 + k);
  hipError_t err = standalone_reserve(sb, (nin + 2) * 8, (nin + 2) * 8);
  if (err != hipSuccess) return set_error(GPDLA_EDEVICE, "log_mvnpdf_low_rank: %s", hipGetErrorString(err));
  double* h = (double*)sb.host;
  std::memcpy(h, y, n * 8);
  std::memcpy(h + n, mu, n * 8);
  std::memcpy(h + 2 * n, d, n * 8);
  std::memcpy(h + 3 * n, M, (size_t)n * k * 8);
  double* dy = (double*)sb.buf;
  double* dmu = dy + n;
  double* dd = dmu + n;
  double* dM = dd + n;
  double* dout = dy + nin;
  int32_t* dst = (int32_t*)(dout + 1);
  err = hipMemcpyAsync(dy, h, nin * 8, hipMemcpyHostToDevice, sb.stream);
  if (err == hipSuccess) err = launch_mvn_single(dy, dmu, dM, dd, n, k, dout, dst, sb.stream);
  if (err == hipSuccess) err = hipMemcpyAsync(h + nin, dout, 16, hipMemcpyDeviceToHost, sb.stream);
  if (err == hipSuccess) err = hipStreamSynchronize(sb.stream);
  if (err != hipSuccess) return set_error(GPDLA_EDEVICE, "log_mvnpdf_low_rank: %s", hipGetErrorString(err));
  *out = h[nin];
  int32_t status = 0;
  std::memcpy(&status, h + nin + 1, 4);
  if (status) return set_error(GPDLA_ENUMERIC, "B = I + M'D^-1M is not positive definite");
  return GPDLA_OK;
}

}  // extern "C"
