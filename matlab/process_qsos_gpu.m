% process_qsos_gpu: process_qsos.m with its per-quasar loop run by the GPU engine.
%
% Same workspace contract as process_qsos.m (README.md:285-305): run set_parameters, set
% training_release, training_set_name, dla_catalog_name, prior_ind, release, test_set_name and
% test_ind, then run this script in place of process_qsos.  It reads the same four files and
% writes the same processed_qsos_<test_set_name>.mat: the 22 variables of process_qsos.m:235-249,
% saved -v7.3.
%
% On the MATLAB path it needs gpdla_mex (matlab/gpdla_mex.c, built with
%   mex -R2018a matlab/gpdla_mex.c -Imatlab -Iinclude -Lgp_dla_detection_amd -lgpdla)
% and the reference's own helpers that process_qsos.m also calls (processed_directory,
% observed_wavelengths).
%
% Optional workspace variables:
%   gpu_device       HIP device index (default 0)
%   likelihood_path  'auto' (default), 'fused', 'panel_gemm', 'fused_i8', 'panel_gemm_i8',
%                    'panel_gemm_i8_24' (INTEGRATION.md section 3)
%   absorption_mode  0 (default) = the reference's absorption(1:n) indexing (process_qsos.m:180,189);
%                    1 = each unmasked pixel paired with its own profile value
%
% The preloaded cells may be single (fitsread's class, read_spec.m:11-31) or double; the engine
% widens single values exactly and computes in double.

if ~exist('gpu_device', 'var'),      gpu_device      = 0;      end
if ~exist('likelihood_path', 'var'), likelihood_path = 'auto'; end
if ~exist('absorption_mode', 'var'), absorption_mode = 0;      end

% ---------------------------------------------------------------- prior catalogue (:3-26)
prior_catalog = load(sprintf('%s/catalog', processed_directory(training_release)));
if ischar(prior_ind)
  prior_ind = eval(prior_ind);          % the index string names prior_catalog, as in the reference
end

prior.z_qsos  = prior_catalog.z_qsos(prior_ind);
prior_dla_ind = prior_catalog.dla_inds(dla_catalog_name);
prior.dla_ind = prior_dla_ind(prior_ind);
prior_z_dlas  = prior_catalog.z_dlas(dla_catalog_name);
prior_z_dlas  = prior_z_dlas(prior_ind);

% a catalogued DLA whose Lyman-alpha line falls below its quasar's Lyman limit is not counted
for i = find(prior.dla_ind)'
  if observed_wavelengths(lya_wavelength, prior_z_dlas{i}) < ...
     observed_wavelengths(lyman_limit,    prior.z_qsos(i))
    prior.dla_ind(i) = false;
  end
end
clear prior_dla_ind prior_z_dlas;

% ---------------------------------------------------- learned model, DLA samples (:28-40)
load(sprintf('%s/learned_qso_model_%s', processed_directory(training_release), training_set_name), ...
     'rest_wavelengths', 'mu', 'M', 'log_omega', 'log_c_0', 'log_tau_0', 'log_beta');
load(sprintf('%s/dla_samples', processed_directory(training_release)), ...
     'offset_samples', 'log_nhi_samples', 'nhi_samples');

% ----------------------------------------------------------- spectra to process (:42-62)
catalog = load(sprintf('%s/catalog', processed_directory(release)));
load(sprintf('%s/preloaded_qsos', processed_directory(release)), ...
     'all_wavelengths', 'all_flux', 'all_noise_variance', 'all_pixel_mask');
if ischar(test_ind)
  test_ind = eval(test_ind);            % the index string names catalog, as in the reference
end

all_wavelengths    =    all_wavelengths(test_ind);
all_flux           =           all_flux(test_ind);
all_noise_variance = all_noise_variance(test_ind);
all_pixel_mask     =     all_pixel_mask(test_ind);
z_qsos             =     catalog.z_qsos(test_ind);
num_quasars        =     numel(z_qsos);

% ------------------------------------------------ DLA prior per quasar (:122-132)
% Among the prior quasars below z_QSO + prior_z_qso_increase, the fraction with a counted DLA.
log_priors_no_dla = nan(num_quasars, 1);
log_priors_dla    = nan(num_quasars, 1);
for quasar_ind = 1:num_quasars
  below       = prior.z_qsos < (z_qsos(quasar_ind) + prior_z_qso_increase);
  n_quasars   = nnz(below);
  n_dlas      = nnz(prior.dla_ind(below));
  log_priors_dla(quasar_ind)    = log(n_dlas)             - log(n_quasars);
  log_priors_no_dla(quasar_ind) = log(n_quasars - n_dlas) - log(n_quasars);
end

% ----------------------------------------------------------- likelihoods on the GPU (:88-212)
% One engine call replaces the loop over quasars: pixel selection, model interpolation, the
% null-model likelihood, every DLA sample's Voigt profile and low-rank likelihood (the parfor of
% :184-198) and the log-mean-exp over samples; z_DLA limits come back with them.
eng = gpdla_mex('create', gpu_device, rest_wavelengths, mu, M, log_omega, ...
                log_c_0, log_tau_0, log_beta, offset_samples, nhi_samples, ...
                num_lines, width, pixel_spacing, min_lambda, max_lambda, ...
                lya_wavelength, lyman_limit, min_z_cut, max_z_cut, ...
                absorption_mode, likelihood_path);
cleanup_engine = onCleanup(@() gpdla_mex('destroy', eng));

tic;
[log_likelihoods_no_dla, sample_log_likelihoods_dla, log_likelihoods_dla, ...
 min_z_dlas, max_z_dlas] = ...
    gpdla_mex('process', eng, all_wavelengths, all_flux, all_noise_variance, ...
              all_pixel_mask, z_qsos);
fprintf('%d quasars x %d DLA samples on the GPU: %0.3fs\n', ...
        num_quasars, numel(offset_samples), toc);
clear cleanup_engine;

% ------------------------------------------------------------ posteriors (:153, 211, 222-232)
log_posteriors_no_dla = log_priors_no_dla + log_likelihoods_no_dla;
log_posteriors_dla    = log_priors_dla    + log_likelihoods_dla;

both_log_posteriors = [log_posteriors_no_dla, log_posteriors_dla];
model_posteriors    = exp(both_log_posteriors - max(both_log_posteriors, [], 2));
model_posteriors    = model_posteriors ./ sum(model_posteriors, 2);
clear both_log_posteriors;

p_no_dlas = model_posteriors(:, 1);
p_dlas    = 1 - p_no_dlas;

% ------------------------------------------------------------------------- save (:234-249)
variables_to_save = {'training_release', 'training_set_name', ...
                     'dla_catalog_name', 'prior_ind', 'release', ...
                     'test_set_name', 'test_ind', 'prior_z_qso_increase', ...
                     'max_z_cut', 'num_lines', 'min_z_dlas', 'max_z_dlas', ...
                     'log_priors_no_dla', 'log_priors_dla', ...
                     'log_likelihoods_no_dla', 'sample_log_likelihoods_dla', ...
                     'log_likelihoods_dla', 'log_posteriors_no_dla', ...
                     'log_posteriors_dla', 'model_posteriors', 'p_no_dlas', ...
                     'p_dlas'};

save(sprintf('%s/processed_qsos_%s', processed_directory(release), test_set_name), ...
     variables_to_save{:}, '-v7.3');
