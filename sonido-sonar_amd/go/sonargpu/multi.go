package sonargpu

// Many stream pairs on one GPU, and one process over several GPUs (include/sonar_gpu.h,
// sonar_align_pairs / sonar_multi_*).  The seams are the same as in sonargpu.go:
//
//	AlignPairs        <- a loop of AlignmentExtractor.ExtractAlignmentFeatures
//	                     (fingerprint/extractors/alignment.go:139) over independent pairs
//	Multi.Fingerprint <- FingerprintGenerator.GenerateFingerprint's STFT + MFCC
//	                     (fingerprint/fingerprint.go:137) with the frames sharded over GPUs
//	Multi.AlignPairs  <- AlignPairs with the pairs sharded over GPUs (records through RCCL)
//
// The pair entries take arrays of stream pointers.  cgo forbids storing Go pointers in C memory
// unless they are pinned, so the slices are pinned with runtime.Pinner (Go 1.21) for the call.
// HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default, at most 32):
// set it to at least the library's pair streams (SONAR_PAIR_STREAMS, default 16) in the
// environment before the first call into the library.  `workers` is the number of pairs in flight
// (<= 0: 128, i.e. 16 streams x batches of 8).

/*
#include <stdlib.h>
#include "sonar_gpu.h"
*/
import "C"

import (
	"fmt"
	"runtime"
	"unsafe"
)

// PairRecord is what ExtractAlignmentFeatures leaves per pair (sonar_pair_record).
type PairRecord struct {
	TemporalOffset, OffsetConfidence, AlignmentSimilarity, AlignmentQuality float64
	Method                                                                   int
	CorrOffsetSeconds, DTWDistance, PeakLag                                  float64
	// Redone: the record came from the single-pair path (SONAR_PAIR_REDONE_TIMEOUT /
	// SONAR_PAIR_REDONE_NONFINITE bits), not from the pair's batch
	Redone int
	Err    error
}

// pairArgs builds the C pointer/length arrays of the pairs' streams, pinning every slice.
func pairArgs(queries, references [][]float64, pin *runtime.Pinner) (qp, rp unsafe.Pointer, nq, nr []C.int64_t,
	err error) {
	n := len(queries)
	if n != len(references) {
		return nil, nil, nil, nil, fmt.Errorf("sonargpu: %d queries vs %d references: %w", n, len(references), ErrInvalid)
	}
	qp = C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0))))
	rp = C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(uintptr(0))))
	qs := unsafe.Slice((**C.double)(qp), n)
	rs := unsafe.Slice((**C.double)(rp), n)
	nq, nr = make([]C.int64_t, n), make([]C.int64_t, n)
	for k := 0; k < n; k++ {
		if len(queries[k]) == 0 || len(references[k]) == 0 {
			C.free(qp)
			C.free(rp)
			return nil, nil, nil, nil, fmt.Errorf("empty signal (pair %d): %w", k, ErrEmpty)
		}
		pin.Pin(&queries[k][0])
		pin.Pin(&references[k][0])
		qs[k], rs[k] = (*C.double)(&queries[k][0]), (*C.double)(&references[k][0])
		nq[k], nr[k] = C.int64_t(len(queries[k])), C.int64_t(len(references[k]))
	}
	return qp, rp, nq, nr, nil
}

func records(recs []C.sonar_pair_record) []PairRecord {
	out := make([]PairRecord, len(recs))
	for k, r := range recs {
		out[k] = PairRecord{
			TemporalOffset: float64(r.temporal_offset), OffsetConfidence: float64(r.offset_confidence),
			AlignmentSimilarity: float64(r.alignment_similarity), AlignmentQuality: float64(r.alignment_quality),
			Method: int(r.method), CorrOffsetSeconds: float64(r.corr_offset_seconds),
			DTWDistance: float64(r.dtw_distance), PeakLag: float64(r.peak_lag), Redone: int(r.flags),
		}
		if r.status != C.SONAR_OK {
			out[k].Err = fmt.Errorf("sonargpu: pair %d failed (%d)", k, int(r.status))
		}
	}
	return out
}

// AlignPairs runs ExtractAlignmentFeatures (music-extractor energy + chroma of both streams, NCC
// of the energies, DTW of the chroma, the scorers) on every pair, `workers` pairs in flight.
func (x *Context) AlignPairs(queries, references [][]float64, sampleRate, stftWindow, hop, featureWindow int,
	maxLagSeconds float64, workers int) ([]PairRecord, error) {
	if len(queries) == 0 {
		return nil, nil
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	qp, rp, nq, nr, err := pairArgs(queries, references, &pin)
	if err != nil {
		return nil, err
	}
	defer C.free(qp)
	defer C.free(rp)
	recs := make([]C.sonar_pair_record, len(queries))
	rc := C.sonar_align_pairs(x.c, C.int64_t(len(queries)), (**C.double)(qp), &nq[0], (**C.double)(rp), &nr[0],
		C.int32_t(sampleRate), C.int32_t(stftWindow), C.int32_t(hop), C.int32_t(featureWindow),
		C.double(maxLagSeconds), C.int32_t(workers), 0, &recs[0])
	return records(recs), x.err(rc)
}

// Multi drives several GPUs from one process: a Context per device and an RCCL communicator.
type Multi struct{ m *C.sonar_multi }

// NewMulti opens the listed devices (HIP ordinals).
func NewMulti(devices []int) (*Multi, error) {
	if len(devices) == 0 {
		return nil, fmt.Errorf("sonargpu: no devices: %w", ErrInvalid)
	}
	ds := make([]C.int32_t, len(devices))
	for i, d := range devices {
		ds[i] = C.int32_t(d)
	}
	var m *C.sonar_multi
	if rc := C.sonar_multi_create(&ds[0], C.int32_t(len(ds)), &m); rc != C.SONAR_OK {
		return nil, fmt.Errorf("sonargpu: sonar_multi_create failed (%d): %w", int(rc), ErrDevice)
	}
	return &Multi{m: m}, nil
}

// Close releases every device context and the communicator.
func (x *Multi) Close() {
	if x.m != nil {
		C.sonar_multi_destroy(x.m)
		x.m = nil
	}
}

func (x *Multi) err(rc C.int) error {
	if rc == C.SONAR_OK {
		return nil
	}
	return fmt.Errorf("%s (%d)", C.GoString(C.sonar_multi_last_error(x.m)), int(rc))
}

// Fingerprint is Context.Fingerprint with the STFT frames sharded over the devices.
func (x *Multi) Fingerprint(pcm []float64, windowSize, hopSize, sampleRate int, p MFCCParams,
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
	if rc := C.sonar_fingerprint_multi(x.m, unsafe.Pointer(&pcm[0]), C.int64_t(len(pcm)), &cfg, out); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	return split(flat, frames, nc), nil
}

// AlignPairs shards the pairs over the devices (contiguous ranges); the records come back
// through one RCCL all-gather.
func (x *Multi) AlignPairs(queries, references [][]float64, sampleRate, stftWindow, hop, featureWindow int,
	maxLagSeconds float64, workers int) ([]PairRecord, error) {
	if len(queries) == 0 {
		return nil, nil
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	qp, rp, nq, nr, err := pairArgs(queries, references, &pin)
	if err != nil {
		return nil, err
	}
	defer C.free(qp)
	defer C.free(rp)
	recs := make([]C.sonar_pair_record, len(queries))
	rc := C.sonar_align_pairs_multi(x.m, C.int64_t(len(queries)), (**C.double)(qp), &nq[0], (**C.double)(rp), &nr[0],
		C.int32_t(sampleRate), C.int32_t(stftWindow), C.int32_t(hop), C.int32_t(featureWindow),
		C.double(maxLagSeconds), C.int32_t(workers), &recs[0])
	return records(recs), x.err(rc)
}

// FingerprintBatch32 is SpectralAnalyzer.ComputeSTFTBatch (fingerprint/analyzers/spectral.go:234-285)
// followed by MFCC.ComputeFrames per signal, on float32 samples (sonar_fingerprint_batch): at
// W = 1024 every signal's frames run in ONE kernel launch.  Returns one F_i x NumCoefficients
// matrix per signal; errors name the first failing signal as ComputeSTFTBatch does.
func (x *Context) FingerprintBatch32(signals [][]float32, windowSize, hopSize, sampleRate int,
	p MFCCParams) ([][][]float32, error) {
	k := len(signals)
	if k == 0 {
		return nil, fmt.Errorf("no signals provided: %w", ErrEmpty)
	}
	var cfg C.sonar_fp_cfg
	C.sonar_fp_cfg_default(&cfg)
	cfg.window_size, cfg.hop_size, cfg.sample_rate = C.int32_t(windowSize), C.int32_t(hopSize), C.int32_t(sampleRate)
	cfg.n_mfcc, cfg.n_filters = C.int32_t(p.NumCoefficients), C.int32_t(p.NumFilters)
	cfg.low_freq, cfg.high_freq, cfg.lifter = C.double(p.LowFreq), C.double(p.HighFreq), C.double(p.LifterCoeff)
	cfg.use_lifter = b2i(p.UseLiftering)
	cfg.flags = C.SONAR_FP_MFCC
	cfg.precision, cfg.pcm_dtype, cfg.out_dtype = C.SONAR_F32, C.SONAR_F32, C.SONAR_F32
	nc := p.NumCoefficients
	if nc <= 0 {
		nc = 13
	}
	var pin runtime.Pinner // the C arrays hold pointers to the Go slices during the call
	defer pin.Unpin()
	pp := C.malloc(C.size_t(k) * C.size_t(unsafe.Sizeof(uintptr(0))))
	defer C.free(pp)
	op := C.calloc(C.size_t(k), C.size_t(unsafe.Sizeof(C.sonar_fp_out{})))
	defer C.free(op)
	ptrs := unsafe.Slice((*unsafe.Pointer)(pp), k)
	outs := unsafe.Slice((*C.sonar_fp_out)(op), k)
	ns := make([]C.int64_t, k)
	flats := make([][]float32, k)
	frames := make([]int, k)
	for i, s := range signals {
		ptrs[i] = nil
		ns[i] = C.int64_t(len(s))
		if len(s) > 0 {
			pin.Pin(&s[0])
			ptrs[i] = unsafe.Pointer(&s[0])
		}
		frames[i] = int(C.sonar_stft_frames(C.int64_t(len(s)), C.int32_t(windowSize), C.int32_t(hopSize)))
		if frames[i] > 0 {
			flats[i] = make([]float32, frames[i]*nc)
			pin.Pin(&flats[i][0])
			outs[i].mfcc = unsafe.Pointer(&flats[i][0])
		}
	}
	if rc := C.sonar_fingerprint_batch(x.c, (*unsafe.Pointer)(pp), &ns[0], C.int32_t(k), &cfg,
		(*C.sonar_fp_out)(op)); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	res := make([][][]float32, k)
	for i := range signals {
		res[i] = make([][]float32, frames[i])
		for f := 0; f < frames[i]; f++ {
			res[i][f] = flats[i][f*nc : (f+1)*nc : (f+1)*nc]
		}
	}
	return res, nil
}
