// Package sonargpu is the cgo shim between the Go library (RyanBlaney/sonido-sonar)
// and libsonar_gpu.so, the MI355X implementation of its per-frame DSP and
// alignment hot path.  It is the "reference-side binding" INTEGRATION.md
// describes: a maintainer drops this directory into the Go module (for
// example as internal/sonargpu) and calls it from the two seams named below.
//
//	GenerateFingerprint   <- fingerprint/fingerprint.go:137 (FingerprintGenerator.GenerateFingerprint)
//	ExtractSpeech         <- fingerprint/extractors/speech.go:135 (SpeechFeatureExtractor.ExtractFeatures)
//	AlignFeatures         <- fingerprint/extractors/alignment.go:139 (AlignmentExtractor.ExtractAlignmentFeatures)
//	DetectFromAudio       <- fingerprint/content_detector.go:72 (ContentDetector.DetectFromAudio)
//	Gallery (compare.go)  <- fingerprint/comparison.go (FingerprintComparator)
//	Fingerprint / DTW / NCC are the lower seams: analyzers/spectral.go:385 + spectral/mfcc.go:167,
//	stats/dtw.go:55, stats/correlation.go:131.
//
// Ownership follows the cgo rules: Go allocates every host slice and passes &s[0];
// the C side owns device memory and its HIP stream inside the Context and keeps
// no Go pointer after a call returns.  A Context is not goroutine-safe (neither are
// the Go objects it replaces); use one per goroutine.
//
// No Go toolchain exists in the build container of this repository, so this file is
// written against include/sonar_gpu.h and has not been compiled there.
package sonargpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../lib -lsonar_gpu -Wl,-rpath,${SRCDIR}/../../lib
#include <stdlib.h>
#include "sonar_gpu.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"unsafe"
)

// Error codes of include/sonar_gpu.h.
var (
	ErrInvalid     = errors.New("sonargpu: invalid argument")
	ErrTooShort    = errors.New("sonargpu: signal too short")
	ErrEmpty       = errors.New("sonargpu: empty input")
	ErrUnsupported = errors.New("sonargpu: unsupported configuration")
	ErrDevice      = errors.New("sonargpu: HIP runtime error")
	ErrNoMem       = errors.New("sonargpu: device allocation failed")
	// ErrPanic: the Go reference panics on this input; the message is the runtime error text
	ErrPanic = errors.New("sonargpu: the reference panics on this input")
)

// Precision of the device arithmetic.
const (
	F32 = int(C.SONAR_F32) // throughput mode (1e-4 relative to the fp64 Go path)
	F64 = int(C.SONAR_F64) // parity mode
)

// Context owns a device, a HIP stream and cached device tables.
type Context struct{ c *C.sonar_ctx }

// NewContext opens device `device` (HIP ordinal).
func NewContext(device int) (*Context, error) {
	var c *C.sonar_ctx
	if rc := C.sonar_create(C.int(device), &c); rc != C.SONAR_OK {
		return nil, fmt.Errorf("sonargpu: sonar_create(%d) failed (%d)", device, int(rc))
	}
	return &Context{c: c}, nil
}

// Close releases the device resources.
func (x *Context) Close() {
	if x.c != nil {
		C.sonar_destroy(x.c)
		x.c = nil
	}
}

// Trim frees the device and pinned host buffers the context (and the worker
// contexts of AlignPairs) cache between calls (sonar_trim); the next call
// allocates again.
func (x *Context) Trim() error {
	return x.err(C.sonar_trim(x.c))
}

// err maps a return code to a Go error carrying the C side's message, which uses
// the reference's own error text ("empty signal", "signal too short for given
// window size and hop size", "empty sequences provided", ...).
func (x *Context) err(rc C.int) error {
	if rc == C.SONAR_OK {
		return nil
	}
	msg := C.GoString(C.sonar_last_error(x.c))
	var base error
	switch rc {
	case C.SONAR_ERR_TOO_SHORT:
		base = ErrTooShort
	case C.SONAR_ERR_EMPTY:
		base = ErrEmpty
	case C.SONAR_ERR_UNSUPPORTED:
		base = ErrUnsupported
	case C.SONAR_ERR_DEVICE:
		base = ErrDevice
	case C.SONAR_ERR_NOMEM:
		base = ErrNoMem
	case C.SONAR_ERR_PANIC:
		base = ErrPanic
	default:
		base = ErrInvalid
	}
	return fmt.Errorf("%s: %w", msg, base)
}

func f64p(s []float64) *C.double {
	if len(s) == 0 {
		return nil
	}
	return (*C.double)(unsafe.Pointer(&s[0]))
}

// rows2 flattens a [][]float64 into one contiguous row-major slice (the one copy
// SURVEY.md section 8(b) budgets for the [][] <-> contiguous conversion).
func rows2(m [][]float64) ([]float64, int) {
	if len(m) == 0 {
		return nil, 0
	}
	d := len(m[0])
	out := make([]float64, 0, len(m)*d)
	for _, r := range m {
		out = append(out, r...)
	}
	return out, d
}

func split(flat []float64, rows, cols int) [][]float64 {
	out := make([][]float64, rows)
	for i := range out {
		out[i] = flat[i*cols : (i+1)*cols : (i+1)*cols]
	}
	return out
}

// Result is a set of named float64 arrays returned by the Go-API mirror entries.
type Result struct {
	Arrays  map[string][]float64
	Shapes  map[string][2]int
	Scalars map[string]float64
}

// Matrix returns a named 2-D result as [][]float64 (e.g. "mfcc").
func (r *Result) Matrix(name string) [][]float64 {
	a, ok := r.Arrays[name]
	if !ok {
		return nil
	}
	s := r.Shapes[name]
	return split(a, s[0], s[1])
}

func (x *Context) collect(res *C.sonar_result) *Result {
	defer C.sonar_result_free(res)
	out := &Result{Arrays: map[string][]float64{}, Shapes: map[string][2]int{}, Scalars: map[string]float64{}}
	n := int(C.sonar_result_count(res))
	for i := 0; i < n; i++ {
		cname := C.sonar_result_name(res, C.int(i))
		name := C.GoString(cname)
		var data *C.double
		var rows, cols C.int64_t
		if C.sonar_result_get(res, cname, &data, &rows, &cols) != C.SONAR_OK {
			continue
		}
		cnt := int(rows) * int(cols)
		vals := make([]float64, cnt)
		if cnt > 0 {
			copy(vals, unsafe.Slice((*float64)(unsafe.Pointer(data)), cnt))
		}
		out.Arrays[name] = vals
		out.Shapes[name] = [2]int{int(rows), int(cols)}
		if cnt == 1 {
			out.Scalars[name] = vals[0]
		}
	}
	return out
}

// FingerprintConfig mirrors fingerprint.FingerprintConfig (fingerprint.go:29-35).
type FingerprintConfig struct {
	WindowSize, HopSize               int
	FeatureWindowSize, FeatureHopSize int // FingerprintConfig.FeatureConfig.{WindowSize,HopSize}
	EnableContentDetect               bool
	Precision                         int
	// ContentConfig (config.ContentAwareConfig) and the rest of AudioData.Metadata, read by
	// ContentDetector.DetectContentType when the content type is unknown
	EnableContentDetection bool
	DefaultContentType     int // SONAR_CT_*
	AutoDetectThreshold    float64
	Genre, Station, URL    string
}

// DefaultFingerprintConfig mirrors DefaultFingerprintConfig (fingerprint.go:70-98).
func DefaultFingerprintConfig() FingerprintConfig {
	var c C.sonar_fingerprint_config
	C.sonar_fingerprint_config_default(&c)
	return FingerprintConfig{WindowSize: int(c.window_size), HopSize: int(c.hop_size),
		FeatureWindowSize: int(c.feature_window_size), FeatureHopSize: int(c.feature_hop_size),
		EnableContentDetect: c.enable_content_detect != 0, Precision: int(c.precision),
		EnableContentDetection: c.acoustic_detection != 0, DefaultContentType: int(c.default_content_type),
		AutoDetectThreshold: float64(c.auto_detect_threshold)}
}

// AcousticFeatures mirrors fingerprint.AcousticFeatures (content_detector.go:104-115).
type AcousticFeatures C.sonar_acoustic_features

// DetectFromAudio runs ContentDetector.DetectFromAudio (content_detector.go:72) on the GPU.
func (x *Context) DetectFromAudio(pcm []float64, sampleRate int, threshold float64) (int, AcousticFeatures, error) {
	var ct C.int32_t
	var f C.sonar_acoustic_features
	if rc := C.sonar_detect_from_audio(x.c, f64p(pcm), C.int64_t(len(pcm)), C.int32_t(sampleRate),
		C.double(threshold), &ct, &f); rc != C.SONAR_OK {
		return 0, AcousticFeatures{}, x.err(rc)
	}
	return int(ct), AcousticFeatures(f), nil
}

// AlignmentStats mirrors stats.AlignmentStats (algorithms/stats/alignment.go:700-707) plus the
// AlignFeatures offset and the trial count.
type AlignmentStats C.sonar_alignment_stats

// AnalyzeAlignmentConsistency runs AlignmentAnalyzer.AnalyzeAlignmentConsistency
// (stats/alignment.go:709) on the GPU; method is the stats.AlignmentMethod value.
func (x *Context) AnalyzeAlignmentConsistency(query, reference [][]float64, sampleRate, method, maxLag, hopSize,
	numTrials int) (AlignmentStats, error) {
	q, dim := rows2(query)
	r, _ := rows2(reference)
	var st C.sonar_alignment_stats
	if rc := C.sonar_alignment_consistency(x.c, f64p(q), C.int64_t(len(query)), f64p(r), C.int64_t(len(reference)),
		C.int32_t(dim), C.int32_t(method), C.int32_t(maxLag), C.int32_t(hopSize), C.int32_t(sampleRate),
		C.int32_t(numTrials), &st); rc != C.SONAR_OK {
		return AlignmentStats{}, x.err(rc)
	}
	return AlignmentStats(st), nil
}

// TruncateToAlignmentPCM mirrors AlignmentExtractor.TruncateToAlignmentPCM
// (extractors/alignment.go:223): the aligned sub-slices of the two streams.
func (x *Context) TruncateToAlignmentPCM(pcm1, pcm2 []float64, sampleRate int, temporalOffset float64) ([]float64,
	[]float64, error) {
	var s1, s2, n C.int64_t
	if rc := C.sonar_truncate_to_alignment(x.c, C.int64_t(len(pcm1)), C.int64_t(len(pcm2)), C.int32_t(sampleRate),
		C.double(temporalOffset), &s1, &s2, &n); rc != C.SONAR_OK {
		return nil, nil, x.err(rc)
	}
	return pcm1[int(s1) : int(s1)+int(n)], pcm2[int(s2) : int(s2)+int(n)], nil
}

// VoiceQuality mirrors speech.VoiceQualityResult (algorithms/speech/voice_quality.go:21-43).
type VoiceQuality C.sonar_voice_quality_result

// AnalyzeVoiceQuality runs VoiceQualityAnalyzer.AnalyzeVoiceQuality (voice_quality.go:56) on
// the GPU; errors carry the Go messages (shorter than one second, fewer than 3 periods).
func (x *Context) AnalyzeVoiceQuality(signal []float64, sampleRate int) (VoiceQuality, error) {
	var q C.sonar_voice_quality_result
	if rc := C.sonar_voice_quality(x.c, f64p(signal), C.int64_t(len(signal)), C.int32_t(sampleRate),
		&q); rc != C.SONAR_OK {
		return VoiceQuality{}, x.err(rc)
	}
	return VoiceQuality(q), nil
}

// GenerateFingerprint runs FingerprintGenerator.GenerateFingerprint's feature path
// (content-type resolution, F1 SampleRate=0 extractor, STFT, features) on the GPU.
// contentType is audioData.Metadata.ContentType.
func (x *Context) GenerateFingerprint(pcm []float64, sampleRate int, contentType string,
	cfg FingerprintConfig) (*Result, error) {
	if len(pcm) == 0 {
		return nil, fmt.Errorf("empty signal: %w", ErrEmpty)
	}
	cc := C.sonar_fingerprint_config{}
	C.sonar_fingerprint_config_default(&cc)
	cc.window_size, cc.hop_size = C.int32_t(cfg.WindowSize), C.int32_t(cfg.HopSize)
	cc.feature_window_size, cc.feature_hop_size = C.int32_t(cfg.FeatureWindowSize), C.int32_t(cfg.FeatureHopSize)
	cc.enable_content_detect = 0
	if cfg.EnableContentDetect {
		cc.enable_content_detect = 1
	}
	cc.precision = C.int32_t(cfg.Precision)
	cc.acoustic_detection = b2i(cfg.EnableContentDetection)
	cc.default_content_type = C.int32_t(cfg.DefaultContentType)
	cc.auto_detect_threshold = C.double(cfg.AutoDetectThreshold)
	for _, m := range []struct {
		s   string
		dst **C.char
	}{{cfg.Genre, &cc.genre}, {cfg.Station, &cc.station}, {cfg.URL, &cc.url}} {
		if m.s != "" {
			*m.dst = C.CString(m.s)
			defer C.free(unsafe.Pointer(*m.dst))
		}
	}
	ct := C.CString(contentType)
	defer C.free(unsafe.Pointer(ct))
	var res *C.sonar_result
	if rc := C.sonar_generate_fingerprint(x.c, f64p(pcm), C.int64_t(len(pcm)), C.int32_t(sampleRate), ct,
		&cc, &res); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	return x.collect(res), nil
}

// FeatureConfig mirrors the config.FeatureConfig fields the speech extractor reads.
type FeatureConfig struct {
	SampleRate, WindowSize, HopSize                          int
	EnableMFCC, EnableSpeechFeatures, EnableTemporalFeatures bool
	MFCCCoefficients                                         int
	Precision                                                int
}

func b2i(b bool) C.int32_t {
	if b {
		return 1
	}
	return 0
}

// ExtractSpeech = NewSpeechFeatureExtractor(&cfg, isNews).ExtractFeatures(STFT(pcm, W, H), pcm, sampleRate).
func (x *Context) ExtractSpeech(pcm []float64, sampleRate, stftWindow, stftHop int, cfg FeatureConfig,
	isNews bool) (*Result, error) {
	var fc C.sonar_feature_config
	C.sonar_feature_config_default(&fc)
	fc.sample_rate, fc.window_size, fc.hop_size = C.int32_t(cfg.SampleRate), C.int32_t(cfg.WindowSize), C.int32_t(cfg.HopSize)
	fc.stft_window_size, fc.stft_hop_size = C.int32_t(stftWindow), C.int32_t(stftHop)
	fc.enable_mfcc, fc.enable_speech_features = b2i(cfg.EnableMFCC), b2i(cfg.EnableSpeechFeatures)
	fc.enable_temporal_features = b2i(cfg.EnableTemporalFeatures)
	fc.mfcc_coefficients, fc.is_news, fc.precision = C.int32_t(cfg.MFCCCoefficients), b2i(isNews), C.int32_t(cfg.Precision)
	var res *C.sonar_result
	if rc := C.sonar_extract_speech_features(x.c, f64p(pcm), C.int64_t(len(pcm)), C.int32_t(sampleRate),
		&fc, &res); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	return x.collect(res), nil
}

// ExtractMusic = NewMusicFeatureExtractor(&cfg).ExtractFeatures(STFT(pcm, W, H), pcm, sampleRate)
// (fingerprint/extractors/music.go:70-583).  Where the reference panics (every signal of 1,536
// samples or more, music.go:403; no energy frame, :383) the error wraps ErrPanic with Go's
// runtime message, and the returned Result holds the arrays computed before that point.  A
// drop-in that must keep the reference's behaviour exactly calls panic(err) there.
func (x *Context) ExtractMusic(pcm []float64, sampleRate, stftWindow, stftHop int, cfg FeatureConfig) (*Result, error) {
	var fc C.sonar_feature_config
	C.sonar_feature_config_default(&fc)
	fc.sample_rate, fc.window_size, fc.hop_size = C.int32_t(cfg.SampleRate), C.int32_t(cfg.WindowSize), C.int32_t(cfg.HopSize)
	fc.stft_window_size, fc.stft_hop_size, fc.precision = C.int32_t(stftWindow), C.int32_t(stftHop), C.int32_t(cfg.Precision)
	var res *C.sonar_result
	rc := C.sonar_extract_music_features(x.c, f64p(pcm), C.int64_t(len(pcm)), C.int32_t(sampleRate), &fc, &res)
	var partial *Result
	if res != nil {
		partial = x.collect(res)
	}
	if rc != C.SONAR_OK {
		return partial, x.err(rc)
	}
	return partial, nil
}

// AlignFeatures = AlignmentExtractor.ExtractAlignmentFeatures on the energy envelopes
// (EnergyFeatures.ShortTimeEnergy) and optional chroma of two fingerprints.
func (x *Context) AlignFeatures(qEnergy, rEnergy []float64, qChroma, rChroma [][]float64,
	qPCMLen, rPCMLen, sampleRate int, featureSampleRate, hop, window int, maxLagSeconds float64) (*Result, error) {
	qc, _ := rows2(qChroma)
	rc2, _ := rows2(rChroma)
	var res *C.sonar_result
	rc := C.sonar_align_features(x.c, f64p(qEnergy), C.int64_t(len(qEnergy)), f64p(rEnergy), C.int64_t(len(rEnergy)),
		f64p(qc), C.int64_t(len(qChroma)), f64p(rc2), C.int64_t(len(rChroma)),
		C.int64_t(qPCMLen), C.int64_t(rPCMLen), C.int32_t(sampleRate), C.int32_t(featureSampleRate),
		C.int32_t(hop), C.int32_t(window), C.double(maxLagSeconds), &res)
	if rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	return x.collect(res), nil
}

// AlignmentMethod values of stats.AlignmentMethod (algorithms/stats/alignment.go:12-17).
const (
	AlignmentDTW              = int(C.SONAR_ALIGN_DTW)
	AlignmentCrossCorrelation = int(C.SONAR_ALIGN_XCORR)
	AlignmentPhaseCorrelation = int(C.SONAR_ALIGN_PHASE)
	AlignmentHybrid           = int(C.SONAR_ALIGN_HYBRID)
)

// AnalyzerAlignFeatures = stats.NewAlignmentAnalyzer(method, maxLag, _, hop, _, _).AlignFeatures(query,
// reference, sampleRate) (algorithms/stats/alignment.go:84-106), including alignWithHybrid's result
// aliasing (:308-337).  The Result holds the AlignmentResult scalars ("offset", "offset_seconds",
// "confidence", "similarity", "alignment_quality", "noise_level", "stability", ...), the
// CrossCorrResult ("correlations", "peak_lag", ...) and the DTWResult ("dtw_distance",
// "dtw_path_query", "dtw_path_reference", "dtw_path_cost") where the method ran them.
func (x *Context) AnalyzerAlignFeatures(query, reference [][]float64, sampleRate, method, maxLag,
	hop int) (*Result, error) {
	q, dim := rows2(query)
	r, _ := rows2(reference)
	var res *C.sonar_result
	if rc := C.sonar_analyzer_align_features(x.c, f64p(q), C.int64_t(len(query)), f64p(r), C.int64_t(len(reference)),
		C.int32_t(dim), C.int32_t(method), C.int32_t(maxLag), C.int32_t(hop), C.int32_t(sampleRate), 0,
		&res); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	return x.collect(res), nil
}

// AlignAudio = AlignmentAnalyzer.AlignAudio (algorithms/stats/alignment.go:108-126): the analyzer's
// RMS energy frames of both signals (extractEnergyFeatures, window / hop), then AlignFeatures.
func (x *Context) AlignAudio(queryPCM, referencePCM []float64, sampleRate, method, maxLag, hop,
	window int) (*Result, error) {
	var res *C.sonar_result
	if rc := C.sonar_align_audio(x.c, f64p(queryPCM), C.int64_t(len(queryPCM)), f64p(referencePCM),
		C.int64_t(len(referencePCM)), C.int32_t(method), C.int32_t(maxLag), C.int32_t(hop), C.int32_t(window),
		C.int32_t(sampleRate), 0, &res); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	return x.collect(res), nil
}

// AlignAudioFiles = AlignmentExtractor.AlignAudioFiles (fingerprint/extractors/alignment.go:489-553)
// for an extractor built by NewAlignmentExtractorWithMaxLag(&FeatureConfig{featureSampleRate, window,
// hop}, _, maxLagSeconds): ShortTimeEnergy of both streams, the Hybrid alignment, and the
// AlignmentFeatures fields ("temporal_offset", "offset_confidence", "alignment_similarity",
// "alignment_quality", "feature_similarity_energy", ...; Method is "energy_correlation").
func (x *Context) AlignAudioFiles(queryPCM, referencePCM []float64, sampleRate, featureSampleRate, hop, window int,
	maxLagSeconds float64) (*Result, error) {
	var res *C.sonar_result
	if rc := C.sonar_align_audio_files(x.c, f64p(queryPCM), C.int64_t(len(queryPCM)), f64p(referencePCM),
		C.int64_t(len(referencePCM)), C.int32_t(sampleRate), C.int32_t(featureSampleRate), C.int32_t(hop),
		C.int32_t(window), C.double(maxLagSeconds), 0, &res); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	return x.collect(res), nil
}

// MFCCParams mirrors spectral.MFCCParams (algorithms/spectral/mfcc.go:27-34).
type MFCCParams struct {
	NumCoefficients, NumFilters int
	LowFreq, HighFreq           float64
	UseLiftering                bool
	LifterCoeff                 float64
}

// Fingerprint is the fused lower seam: SpectralAnalyzer.ComputeSTFTWithWindow(pcm, W, H, Hann)
// followed by NewMFCCWithParams(sampleRate, p).ComputeFrames(|X|) — one kernel, the STFT is
// never materialised.  Returns F x NumCoefficients.
func (x *Context) Fingerprint(pcm []float64, windowSize, hopSize, sampleRate int, p MFCCParams,
	precision int) ([][]float64, error) {
	var cfg C.sonar_fp_cfg
	C.sonar_fp_cfg_default(&cfg)
	cfg.window_size, cfg.hop_size, cfg.sample_rate = C.int32_t(windowSize), C.int32_t(hopSize), C.int32_t(sampleRate)
	cfg.n_mfcc, cfg.n_filters = C.int32_t(p.NumCoefficients), C.int32_t(p.NumFilters)
	cfg.low_freq, cfg.high_freq, cfg.lifter = C.double(p.LowFreq), C.double(p.HighFreq), C.double(p.LifterCoeff)
	cfg.use_lifter = b2i(p.UseLiftering)
	cfg.flags = C.SONAR_FP_MFCC
	cfg.precision, cfg.pcm_dtype, cfg.out_dtype = C.int32_t(precision), C.SONAR_F64, C.SONAR_F64
	frames := int(C.sonar_stft_frames(C.int64_t(len(pcm)), C.int32_t(windowSize), C.int32_t(hopSize)))
	if frames <= 0 {
		return nil, fmt.Errorf("signal too short for given window size and hop size: %w", ErrTooShort)
	}
	nc := p.NumCoefficients
	if nc <= 0 {
		nc = 13
	}
	flat := make([]float64, frames*nc)
	var pin runtime.Pinner
	defer pin.Unpin()
	out := mfccOut(&pin, flat)
	defer C.free(unsafe.Pointer(out))
	if rc := C.sonar_fingerprint(x.c, unsafe.Pointer(&pcm[0]), C.int64_t(len(pcm)), &cfg, out); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	return split(flat, frames, nc), nil
}

// Spectrogram mirrors the per-frame arrays of analyzers.SpectrogramResult
// (fingerprint/analyzers/spectral.go:19-25): Magnitude, Phase and Complex, F x (W/2+1).
type Spectrogram struct {
	Magnitude [][]float64
	Phase     [][]float64
	Complex   [][]complex128
}

// ComputeSTFT is SpectralAnalyzer.ComputeSTFTWithWindow (spectral.go:385) on the GPU, float64:
// the window is {Normalize, Symmetric} like spectral.go:415; frames that Go skips stay zero.
// The complex128 rows are filled in place (Go lays complex128 out as (re, im) float64 pairs,
// which is the C ABI's interleaved SONAR_FP_COMPLEX layout).
func (x *Context) ComputeSTFT(pcm []float64, windowSize, hopSize, windowType int) (*Spectrogram, error) {
	if len(pcm) == 0 {
		return nil, fmt.Errorf("empty signal: %w", ErrEmpty)
	}
	frames := int(C.sonar_stft_frames(C.int64_t(len(pcm)), C.int32_t(windowSize), C.int32_t(hopSize)))
	if frames <= 0 {
		return nil, fmt.Errorf("signal too short for given window size and hop size: %w", ErrTooShort)
	}
	var cfg C.sonar_fp_cfg
	C.sonar_fp_cfg_default(&cfg)
	cfg.window_size, cfg.hop_size, cfg.window_type = C.int32_t(windowSize), C.int32_t(hopSize), C.int32_t(windowType)
	cfg.flags = C.SONAR_FP_MAGNITUDE | C.SONAR_FP_PHASE | C.SONAR_FP_COMPLEX
	cfg.precision, cfg.pcm_dtype, cfg.out_dtype = C.SONAR_F64, C.SONAR_F64, C.SONAR_F64
	k := windowSize/2 + 1
	mag, ph := make([]float64, frames*k), make([]float64, frames*k)
	cx := make([]complex128, frames*k)
	// the output struct holds Go pointers: pinned for the call (cgo's check rejects a Go pointer to
	// unpinned Go pointers), the struct itself in C memory
	var pin runtime.Pinner
	defer pin.Unpin()
	pin.Pin(&mag[0])
	pin.Pin(&ph[0])
	pin.Pin(&cx[0])
	out := (*C.sonar_fp_out)(C.calloc(1, C.size_t(unsafe.Sizeof(C.sonar_fp_out{}))))
	defer C.free(unsafe.Pointer(out))
	out.magnitude, out.phase, out.complex = unsafe.Pointer(&mag[0]), unsafe.Pointer(&ph[0]), unsafe.Pointer(&cx[0])
	if rc := C.sonar_fingerprint(x.c, unsafe.Pointer(&pcm[0]), C.int64_t(len(pcm)), &cfg, out); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	s := &Spectrogram{Magnitude: split(mag, frames, k), Phase: split(ph, frames, k),
		Complex: make([][]complex128, frames)}
	for t := range s.Complex {
		s.Complex[t] = cx[t*k : (t+1)*k]
	}
	return s, nil
}

// FingerprintDecoded is Fingerprint fed by the decoder's raw output instead of AudioData.PCM:
// `output` is the ffmpeg "-f f64le" byte stream (transcode/decoder.go:709) that
// Decoder.bytesToFloat64 (decoder.go:850-871) would walk into a []float64.  The bytes cross
// PCIe through pinned slots (HOST_CONVERT rounds them to float32 on the way, half the bytes),
// so the []float64 copy of the stream is never built.  Float32 throughput mode only.
func (x *Context) FingerprintDecoded(output []byte, windowSize, hopSize, sampleRate int, p MFCCParams) ([][]float64,
	error) {
	if len(output) < 8 {
		return nil, fmt.Errorf("no audio samples decoded: %w", ErrEmpty)
	}
	var cfg C.sonar_fp_cfg
	C.sonar_fp_cfg_default(&cfg)
	cfg.window_size, cfg.hop_size, cfg.sample_rate = C.int32_t(windowSize), C.int32_t(hopSize), C.int32_t(sampleRate)
	cfg.n_mfcc, cfg.n_filters = C.int32_t(p.NumCoefficients), C.int32_t(p.NumFilters)
	cfg.low_freq, cfg.high_freq, cfg.lifter = C.double(p.LowFreq), C.double(p.HighFreq), C.double(p.LifterCoeff)
	cfg.use_lifter = b2i(p.UseLiftering)
	cfg.flags = C.SONAR_FP_MFCC
	cfg.precision, cfg.pcm_dtype, cfg.out_dtype = C.SONAR_F32, C.SONAR_F32, C.SONAR_F64
	frames := int(C.sonar_stft_frames(C.int64_t(len(output)/8), C.int32_t(windowSize), C.int32_t(hopSize)))
	if frames <= 0 {
		return nil, fmt.Errorf("signal too short for given window size and hop size: %w", ErrTooShort)
	}
	nc := p.NumCoefficients
	if nc <= 0 {
		nc = 13
	}
	flat := make([]float64, frames*nc)
	var pin runtime.Pinner
	defer pin.Unpin()
	out := mfccOut(&pin, flat)
	defer C.free(unsafe.Pointer(out))
	if rc := C.sonar_fingerprint_f64le(x.c, unsafe.Pointer(&output[0]), C.int64_t(len(output)),
		C.SONAR_INGEST_HOST_CONVERT, &cfg, out); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	return split(flat, frames, nc), nil
}

// DTWResult mirrors stats.DTWResult + AlignPoint (algorithms/stats/dtw.go:17-34).
type DTWResult struct {
	Distance   float64
	PathQuery  []int
	PathRef    []int
	PathCost   []float64
	CostMatrix [][]float64 // nil unless wantCost (costMatrix[1:], dtw.go:96)
}

// DTW = NewDTWAlignment().Align(q, r) with the Euclidean distance and symmetric2 step;
// band < 0 disables the Sakoe-Chiba window.
func (x *Context) DTW(q, r [][]float64, band int, wantCost bool) (*DTWResult, error) {
	if len(q) == 0 || len(r) == 0 {
		return nil, fmt.Errorf("empty sequences provided: %w", ErrEmpty)
	}
	qf, d := rows2(q)
	rf, _ := rows2(r)
	cap := len(q) + len(r)
	pq, pr := make([]C.int32_t, cap), make([]C.int32_t, cap)
	pc := make([]float64, cap)
	var dist C.double
	var plen C.int64_t
	var cost []float64
	var costp *C.double
	if wantCost {
		cost = make([]float64, len(q)*(len(r)+1))
		costp = f64p(cost)
	}
	rc := C.sonar_dtw(x.c, f64p(qf), C.int64_t(len(q)), f64p(rf), C.int64_t(len(r)), C.int32_t(d), C.int32_t(band),
		&dist, &pq[0], &pr[0], f64p(pc), &plen, costp, 0)
	if rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	res := &DTWResult{Distance: float64(dist), PathQuery: make([]int, plen), PathRef: make([]int, plen),
		PathCost: pc[:plen]}
	for i := 0; i < int(plen); i++ {
		res.PathQuery[i], res.PathRef[i] = int(pq[i]), int(pr[i])
	}
	if wantCost {
		res.CostMatrix = split(cost, len(q), len(r)+1)
	}
	return res, nil
}

// CorrelationResult mirrors the fields of stats.CorrelationResult (correlation.go:44-70) the alignment code reads.
type CorrelationResult struct {
	Correlations                                  []float64
	PeakCorrelation                               float64
	PeakLag, PeakIndex                            int
	PValue, SNR, Sharpness, SecondPeak, PSL       float64
	OverlapLength                                 int
}

// NCC = CrossCorrelation{NormalizedCrossCorrelation, TimeDomain, maxLag}.Compute(s1, s2).
func (x *Context) NCC(s1, s2 []float64, maxLag int) (*CorrelationResult, error) {
	if len(s1) == 0 || len(s2) == 0 {
		return nil, fmt.Errorf("empty signals provided: %w", ErrEmpty)
	}
	L := maxLag
	if len(s1)-1 < L {
		L = len(s1) - 1
	}
	if len(s2)-1 < L {
		L = len(s2) - 1
	}
	if L < 0 {
		L = 0
	}
	corr := make([]float64, 2*L+1)
	var m [10]float64
	if rc := C.sonar_ncc(x.c, f64p(s1), C.int64_t(len(s1)), f64p(s2), C.int64_t(len(s2)), C.int32_t(maxLag),
		f64p(corr), (*C.double)(unsafe.Pointer(&m[0])), 0); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	return &CorrelationResult{Correlations: corr, PeakCorrelation: m[0], PeakLag: int(m[1]), PeakIndex: int(m[2]),
		PValue: m[3], SNR: m[4], Sharpness: m[5], SecondPeak: m[6], PSL: m[7], OverlapLength: int(m[8])}, nil
}

// mfccOut is a sonar_fp_out in C memory whose mfcc field points at flat, pinned by pin for the
// call: cgo rejects a Go struct holding Go pointers, and C memory may hold a Go pointer only while
// it is pinned.  The caller frees the struct (C.free) and unpins.
func mfccOut(pin *runtime.Pinner, flat []float64) *C.sonar_fp_out {
	out := (*C.sonar_fp_out)(C.calloc(1, C.size_t(unsafe.Sizeof(C.sonar_fp_out{}))))
	pin.Pin(&flat[0])
	out.mfcc = unsafe.Pointer(&flat[0])
	return out
}
