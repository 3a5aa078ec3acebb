% process_qsos_gpu.m -- the GPU engine in place of process_qsos.m's per-quasar loop.
%
% Same workspace contract as process_qsos.m (README.md:285-305): run set_parameters, set
% training_release, training_set_name, dla_catalog_name, prior_ind, release, test_set_name and
% test_ind, then run this script instead of process_qsos.
%
% Steps kept from process_qsos.m, unchanged:  loading the prior catalogue, the learned model, the
% DLA samples and the preloaded spectra (process_qsos.m:1-63); the prior counts (:122-132); the
% posteriors and the save (:222-249).  This file covers what changes: the loop over quasars with
% its parfor over DLA samples (:88-220), which becomes one gpdla_mex engine call (matlab/gpdla_mex.c,
% built with  mex -R2018a matlab/gpdla_mex.c -Iinclude -Lgp_dla_detection_amd -lgpdla).
%
% Inputs from the kept loading steps: rest_wavelengths, mu, M, log_omega, log_c_0, log_tau_0,
% log_beta, offset_samples, nhi_samples, all_wavelengths, all_flux, all_noise_variance,
% all_pixel_mask, z_qsos (each restricted to test_ind as process_qsos.m:57-61 does).

if ~exist('gpu_device', 'var'), gpu_device = 0; end
if ~exist('likelihood_path', 'var'), likelihood_path = 'auto'; end   % see INTEGRATION.md section 3
if ~exist('absorption_mode', 'var'), absorption_mode = 0; end        % 0 = reference quirk (:180,189)

eng = gpdla_mex('create', gpu_device, rest_wavelengths, mu, M, log_omega, ...
                log_c_0, log_tau_0, log_beta, offset_samples, nhi_samples, ...
                num_lines, width, pixel_spacing, min_lambda, max_lambda, ...
                lya_wavelength, lyman_limit, min_z_cut, max_z_cut, ...
                absorption_mode, likelihood_path);
cleanup_engine = onCleanup(@() gpdla_mex('destroy', eng));

tic;
[log_likelihoods_no_dla, sample_log_likelihoods_dla, log_likelihoods_dla, ...
 min_z_dlas, max_z_dlas, num_pixels] = ...
    gpdla_mex('process', eng, all_wavelengths, all_flux, all_noise_variance, ...
              all_pixel_mask, z_qsos);
fprintf('%d quasars x %d DLA samples on the GPU: %0.3fs\n', ...
        numel(z_qsos), numel(offset_samples), toc);
clear cleanup_engine;

% log_priors_no_dla / log_priors_dla: process_qsos.m:122-132 over the prior catalogue.
% log_posteriors_*, model_posteriors, p_no_dlas, p_dlas and the -v7.3 save: process_qsos.m:222-249.
