/* layout.c -- the public structs of include/sonar_gpu.h as a C99 compiler lays them out
 * (cgo compiles the sonar_gpu.h preamble of go/sonargpu/sonargpu.go as C, as here).
 * Prints one "struct <name> <sizeof>" line per struct and one "field <struct>.<member> <offset>"
 * line per member; tests/test_abi_cpu.py compares them with the ctypes mirrors in
 * sonido-sonar_amd/sonar/_abi.py.  The sizes are also pinned at compile time (C99 form of a
 * static assertion: a negative array size), so a header change that moves a layout fails to build.
 * Test infrastructure; build: make -C tests/c_abi (gcc -std=c99 -Wall -Wextra -Werror -pedantic). */
#include <stddef.h>
#include <stdio.h>

#include "sonar_gpu.h"

#define PIN(T, n) typedef char pin_##T[(sizeof(T) == (n)) ? 1 : -1]
#define S(T) printf("struct %s %zu\n", #T, sizeof(T))
#define F(T, m) printf("field %s.%s %zu\n", #T, #m, offsetof(T, m))

PIN(sonar_fp_cfg, 104);
PIN(sonar_fp_out, 120);
PIN(sonar_formant_frame, 176);
PIN(sonar_voice_quality_result, 96);
PIN(sonar_fingerprint_config, 72);
PIN(sonar_feature_config, 48);
PIN(sonar_alignment_stats, 56);
PIN(sonar_acoustic_features, 80);
PIN(sonar_fp_features, 272);
PIN(sonar_compare_cfg, 24);
PIN(sonar_similarity, 136);
PIN(sonar_match, 152);
PIN(sonar_pair_record, 72);

int main(void) {
  S(sonar_fp_cfg);
  F(sonar_fp_cfg, window_size); F(sonar_fp_cfg, hop_size); F(sonar_fp_cfg, window_type);
  F(sonar_fp_cfg, sample_rate); F(sonar_fp_cfg, n_mfcc); F(sonar_fp_cfg, n_filters);
  F(sonar_fp_cfg, filterbank); F(sonar_fp_cfg, use_lifter); F(sonar_fp_cfg, low_freq);
  F(sonar_fp_cfg, high_freq); F(sonar_fp_cfg, lifter); F(sonar_fp_cfg, mfcc_input_power);
  F(sonar_fp_cfg, energy_window); F(sonar_fp_cfg, energy_hop); F(sonar_fp_cfg, preemph_alpha);
  F(sonar_fp_cfg, flags); F(sonar_fp_cfg, precision); F(sonar_fp_cfg, pcm_dtype);
  F(sonar_fp_cfg, out_dtype); F(sonar_fp_cfg, device_ptrs);

  S(sonar_fp_out);
  F(sonar_fp_out, mfcc); F(sonar_fp_out, magnitude); F(sonar_fp_out, centroid); F(sonar_fp_out, rolloff);
  F(sonar_fp_out, bandwidth); F(sonar_fp_out, flatness); F(sonar_fp_out, crest); F(sonar_fp_out, slope);
  F(sonar_fp_out, flux); F(sonar_fp_out, low_ratio); F(sonar_fp_out, high_ratio); F(sonar_fp_out, zcr);
  F(sonar_fp_out, energy); F(sonar_fp_out, complex); F(sonar_fp_out, phase);

  S(sonar_formant_frame);
  F(sonar_formant_frame, status); F(sonar_formant_frame, n_formants); F(sonar_formant_frame, frequency);
  F(sonar_formant_frame, bandwidth); F(sonar_formant_frame, amplitude); F(sonar_formant_frame, confidence);
  F(sonar_formant_frame, vocal_tract_length); F(sonar_formant_frame, quality); F(sonar_formant_frame, gain);
  F(sonar_formant_frame, residual_energy); F(sonar_formant_frame, stable); F(sonar_formant_frame, lpc_order);

  S(sonar_voice_quality_result);
  F(sonar_voice_quality_result, jitter); F(sonar_voice_quality_result, shimmer);
  F(sonar_voice_quality_result, hnr); F(sonar_voice_quality_result, noise_measure);
  F(sonar_voice_quality_result, f0_stability); F(sonar_voice_quality_result, amplitude_stability);
  F(sonar_voice_quality_result, voicing_strength); F(sonar_voice_quality_result, overall_quality);
  F(sonar_voice_quality_result, num_periods); F(sonar_voice_quality_result, mean_f0);
  F(sonar_voice_quality_result, f0_range); F(sonar_voice_quality_result, analysis_quality);

  S(sonar_fingerprint_config);
  F(sonar_fingerprint_config, window_size); F(sonar_fingerprint_config, hop_size);
  F(sonar_fingerprint_config, feature_window_size); F(sonar_fingerprint_config, feature_hop_size);
  F(sonar_fingerprint_config, enable_content_detect); F(sonar_fingerprint_config, window_type);
  F(sonar_fingerprint_config, precision); F(sonar_fingerprint_config, acoustic_detection);
  F(sonar_fingerprint_config, default_content_type); F(sonar_fingerprint_config, auto_detect_threshold);
  F(sonar_fingerprint_config, genre); F(sonar_fingerprint_config, station); F(sonar_fingerprint_config, url);

  S(sonar_feature_config);
  F(sonar_feature_config, sample_rate); F(sonar_feature_config, window_size); F(sonar_feature_config, hop_size);
  F(sonar_feature_config, stft_window_size); F(sonar_feature_config, stft_hop_size);
  F(sonar_feature_config, window_type); F(sonar_feature_config, enable_mfcc);
  F(sonar_feature_config, enable_speech_features); F(sonar_feature_config, enable_temporal_features);
  F(sonar_feature_config, mfcc_coefficients); F(sonar_feature_config, is_news); F(sonar_feature_config, precision);

  S(sonar_alignment_stats);
  F(sonar_alignment_stats, mean_offset); F(sonar_alignment_stats, stddev_offset);
  F(sonar_alignment_stats, median_offset); F(sonar_alignment_stats, offset_range);
  F(sonar_alignment_stats, consistency); F(sonar_alignment_stats, offset); F(sonar_alignment_stats, trials);

  S(sonar_acoustic_features);
  F(sonar_acoustic_features, zero_crossing_rate); F(sonar_acoustic_features, spectral_centroid);
  F(sonar_acoustic_features, energy_variance); F(sonar_acoustic_features, silence_ratio);
  F(sonar_acoustic_features, harmonic_ratio); F(sonar_acoustic_features, low_freq_energy);
  F(sonar_acoustic_features, high_freq_energy); F(sonar_acoustic_features, dynamic_range);
  F(sonar_acoustic_features, temporal_stability); F(sonar_acoustic_features, classification_confidence);

  S(sonar_fp_features);
  F(sonar_fp_features, id); F(sonar_fp_features, present); F(sonar_fp_features, content_type);
  F(sonar_fp_features, duration_seconds); F(sonar_fp_features, mfcc); F(sonar_fp_features, mfcc_frames);
  F(sonar_fp_features, mfcc_coeffs); F(sonar_fp_features, chroma); F(sonar_fp_features, chroma_frames);
  F(sonar_fp_features, chroma_bins); F(sonar_fp_features, spectral_centroid);
  F(sonar_fp_features, n_spectral_centroid); F(sonar_fp_features, spectral_rolloff);
  F(sonar_fp_features, n_spectral_rolloff); F(sonar_fp_features, spectral_flux);
  F(sonar_fp_features, n_spectral_flux); F(sonar_fp_features, dynamic_range);
  F(sonar_fp_features, silence_ratio); F(sonar_fp_features, onset_density); F(sonar_fp_features, rms_energy);
  F(sonar_fp_features, n_rms_energy); F(sonar_fp_features, speech_rate); F(sonar_fp_features, vocal_tract_length);
  F(sonar_fp_features, voicing_probability); F(sonar_fp_features, n_voicing_probability);
  F(sonar_fp_features, harmonic_ratio); F(sonar_fp_features, n_harmonic_ratio);
  F(sonar_fp_features, pitch_estimate); F(sonar_fp_features, n_pitch_estimate);
  F(sonar_fp_features, feature_weights);

  S(sonar_compare_cfg);
  F(sonar_compare_cfg, similarity_threshold); F(sonar_compare_cfg, max_candidates);
  F(sonar_compare_cfg, enable_detailed_metrics); F(sonar_compare_cfg, enable_content_filter);
  F(sonar_compare_cfg, method);

  S(sonar_similarity);
  F(sonar_similarity, overall_similarity); F(sonar_similarity, feature_similarity);
  F(sonar_similarity, confidence); F(sonar_similarity, feature_distances);
  F(sonar_similarity, data_availability); F(sonar_similarity, feature_coverage);
  F(sonar_similarity, temporal_alignment); F(sonar_similarity, noise_level);
  F(sonar_similarity, dynamic_range_match); F(sonar_similarity, spectral_coherence);
  F(sonar_similarity, distance_mask); F(sonar_similarity, content_type_match);
  F(sonar_similarity, has_quality); F(sonar_similarity, status);

  S(sonar_match);
  F(sonar_match, candidate); F(sonar_match, rank); F(sonar_match, match_type); F(sonar_match, similarity);
  S(sonar_pair_record);
  F(sonar_pair_record, temporal_offset); F(sonar_pair_record, offset_confidence);
  F(sonar_pair_record, alignment_similarity); F(sonar_pair_record, alignment_quality);
  F(sonar_pair_record, method); F(sonar_pair_record, corr_offset_seconds); F(sonar_pair_record, dtw_distance);
  F(sonar_pair_record, peak_lag); F(sonar_pair_record, status); F(sonar_pair_record, flags);
  return 0;
}
