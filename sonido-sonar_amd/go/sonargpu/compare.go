package sonargpu

// FingerprintComparator seam (fingerprint/comparison.go): a device gallery of fingerprint
// records plus batched Compare / FindBestMatches.  The maintainer's FingerprintComparator
// keeps one Gallery, adds each *AudioFingerprint once (Features -> CompareInput below) and
// answers Compare (:133), BatchCompare (:1107) and FindBestMatches (:197) from it.
//
// Written against include/sonar_gpu.h; not compiled here (no Go toolchain in the image).

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

// CompareInput is what the comparator reads from one AudioFingerprint.  Nil slices and
// nil sub-structs keep their meaning (Has* = the sub-struct pointer is non-nil).
type CompareInput struct {
	ID          string
	ContentType string
	Duration    float64 // AudioFingerprint.Duration.Seconds()
	HasFeatures bool
	MFCC        [][]float64 // nil = nil slice
	Chroma      [][]float64

	HasSpectral                                 bool
	SpectralCentroid, SpectralRolloff, SpectralFlux []float64

	HasTemporal                               bool
	DynamicRange, SilenceRatio, OnsetDensity  float64
	RMSEnergy                                 []float64

	HasSpeech                     bool
	SpeechRate, VocalTractLength  float64
	VoicingProbability            []float64

	HasHarmonic                   bool
	HarmonicRatio, PitchEstimate  []float64

	FeatureWeights map[string]float64 // Metadata["feature_weights"] when it is a map[string]float64
}

// CompareConfig mirrors config.ComparisonConfig.
type CompareConfig struct {
	SimilarityThreshold   float64
	Method                string
	MaxCandidates         int
	EnableDetailedMetrics bool
	EnableContentFilter   bool
}

// Similarity mirrors SimilarityResult (ProcessingTime and Metadata stay Go-side).
type Similarity struct {
	OverallSimilarity, FeatureSimilarity, Confidence float64
	ContentTypeMatch                                 bool
	FeatureDistances                                 map[string]float64
	Quality                                          *C.sonar_similarity // nil unless detailed metrics
	Skipped                                          bool                // same ID (BatchCompare drops it)
}

var fdKeys = []string{"mfcc", "spectral", "chroma", "temporal", "speech", "harmonic"}

// Gallery owns the device records of the fingerprints added so far.
type Gallery struct {
	g      *C.sonar_gallery
	x      *Context
	ids    map[string]int64
	cts    map[string]int32
	Inputs []*CompareInput
}

func (x *Context) NewGallery() (*Gallery, error) {
	var g *C.sonar_gallery
	if rc := C.sonar_gallery_create(x.c, &g); rc != 0 {
		return nil, x.err(rc)
	}
	cts := map[string]int32{"music": 0, "news": 1, "sports": 2, "talk": 3, "mixed": 4, "unknown": 5}
	return &Gallery{g: g, x: x, ids: map[string]int64{}, cts: cts}, nil
}

func (g *Gallery) Close() { C.sonar_gallery_destroy(g.g) }

func (g *Gallery) code(ct string) int32 {
	if c, ok := g.cts[ct]; ok {
		return c
	}
	c := int32(len(g.cts) + 1)
	g.cts[ct] = c
	return c
}

func (g *Gallery) id(s string) int64 {
	if v, ok := g.ids[s]; ok {
		return v
	}
	v := int64(len(g.ids))
	g.ids[s] = v
	return v
}

// Add summarises the fingerprints on the device and returns the index of the first.
func (g *Gallery) Add(fps []*CompareInput, keepSequences bool) (int64, error) {
	recs := make([]C.sonar_fp_features, len(fps))
	var pins runtime.Pinner // C reads the Go slices during the call only
	defer pins.Unpin()
	vec := func(s []float64) (*C.double, C.int64_t) {
		if len(s) == 0 {
			return nil, 0
		}
		pins.Pin(&s[0])
		return (*C.double)(unsafe.Pointer(&s[0])), C.int64_t(len(s))
	}
	for i, f := range fps {
		r := &recs[i]
		r.id = C.int64_t(g.id(f.ID))
		r.content_type = C.int32_t(g.code(f.ContentType))
		r.duration_seconds = C.double(f.Duration)
		var p C.uint32_t
		if f.HasFeatures {
			p |= C.SONAR_FEAT_FEATURES
			if f.MFCC != nil {
				p |= C.SONAR_FEAT_MFCC
				flat, cols := rowsPad(f.MFCC) // rows padded to len(mfcc[0]) with 0 (comparison.go:784-789)
				r.mfcc, _ = vec(flat)
				r.mfcc_frames, r.mfcc_coeffs = C.int64_t(len(f.MFCC)), C.int32_t(cols)
			}
			if f.Chroma != nil {
				p |= C.SONAR_FEAT_CHROMA
				flat, cols := rowsPad(f.Chroma) // chroma rows are len(chroma[0]) wide in practice
				r.chroma, _ = vec(flat)
				r.chroma_frames, r.chroma_bins = C.int64_t(len(f.Chroma)), C.int32_t(cols)
			}
			if f.HasSpectral {
				p |= C.SONAR_FEAT_SPECTRAL
				r.spectral_centroid, r.n_spectral_centroid = vec(f.SpectralCentroid)
				r.spectral_rolloff, r.n_spectral_rolloff = vec(f.SpectralRolloff)
				r.spectral_flux, r.n_spectral_flux = vec(f.SpectralFlux)
			}
			if f.HasTemporal {
				p |= C.SONAR_FEAT_TEMPORAL
				r.dynamic_range, r.silence_ratio, r.onset_density =
					C.double(f.DynamicRange), C.double(f.SilenceRatio), C.double(f.OnsetDensity)
				r.rms_energy, r.n_rms_energy = vec(f.RMSEnergy)
			}
			if f.HasSpeech {
				p |= C.SONAR_FEAT_SPEECH
				r.speech_rate, r.vocal_tract_length = C.double(f.SpeechRate), C.double(f.VocalTractLength)
				r.voicing_probability, r.n_voicing_probability = vec(f.VoicingProbability)
			}
			if f.HasHarmonic {
				p |= C.SONAR_FEAT_HARMONIC
				r.harmonic_ratio, r.n_harmonic_ratio = vec(f.HarmonicRatio)
				r.pitch_estimate, r.n_pitch_estimate = vec(f.PitchEstimate)
			}
		}
		if f.FeatureWeights != nil {
			p |= C.SONAR_FEAT_WEIGHTS
			for k, name := range fdKeys {
				r.feature_weights[k] = C.double(f.FeatureWeights[name]) // missing key -> 0
			}
		}
		r.present = p
	}
	var first C.int64_t
	var rp *C.sonar_fp_features
	if len(recs) > 0 {
		rp = &recs[0]
	}
	if rc := C.sonar_gallery_add(g.g, rp, C.int32_t(len(recs)), b2i(keepSequences), 0, &first); rc != 0 {
		return 0, g.x.err(rc)
	}
	g.Inputs = append(g.Inputs, fps...)
	return int64(first), nil
}

// rowsPad flattens rows to len(m[0]) columns: shorter rows are zero-padded, longer truncated.
func rowsPad(m [][]float64) ([]float64, int) {
	if len(m) == 0 {
		return nil, 0
	}
	d := len(m[0])
	out := make([]float64, len(m)*d)
	for i, r := range m {
		copy(out[i*d:(i+1)*d], r)
	}
	return out, d
}

func cfgOf(c CompareConfig) C.sonar_compare_cfg {
	m := map[string]C.int32_t{"auto": 0, "fast": 1, "precise": 2}
	return C.sonar_compare_cfg{similarity_threshold: C.double(c.SimilarityThreshold),
		max_candidates: C.int32_t(c.MaxCandidates), enable_detailed_metrics: b2i(c.EnableDetailedMetrics),
		enable_content_filter: b2i(c.EnableContentFilter), method: m[c.Method]}
}

func simOf(s *C.sonar_similarity) Similarity {
	out := Similarity{OverallSimilarity: float64(s.overall_similarity),
		FeatureSimilarity: float64(s.feature_similarity), Confidence: float64(s.confidence),
		ContentTypeMatch: s.content_type_match != 0, FeatureDistances: map[string]float64{},
		Skipped: s.status == 1}
	for k, name := range fdKeys {
		if s.distance_mask&(1<<uint(k)) != 0 {
			out.FeatureDistances[name] = float64(s.feature_distances[k])
		}
	}
	if s.has_quality != 0 {
		q := *s
		out.Quality = &q
	}
	return out
}

// BatchCompare: every query against every candidate (gallery indices), out[q][c].
func (g *Gallery) BatchCompare(queries, candidates []int64, cfg CompareConfig) ([][]Similarity, error) {
	c := cfgOf(cfg)
	nq, nc := len(queries), len(candidates)
	buf := make([]C.sonar_similarity, nq*nc+1)
	var qp, cp *C.int64_t
	if nq > 0 {
		qp = (*C.int64_t)(unsafe.Pointer(&queries[0]))
	}
	if nc > 0 {
		cp = (*C.int64_t)(unsafe.Pointer(&candidates[0]))
	}
	if rc := C.sonar_compare(g.g, qp, C.int64_t(nq), cp, C.int64_t(nc), &c, &buf[0], 0); rc != 0 {
		return nil, g.x.err(rc)
	}
	out := make([][]Similarity, nq)
	for q := range out {
		out[q] = make([]Similarity, nc)
		for j := range out[q] {
			out[q][j] = simOf(&buf[q*nc+j])
		}
	}
	return out, nil
}

// Match mirrors fingerprint.Match (the candidate is a gallery index).
type Match struct {
	Candidate  int64
	Rank       int
	MatchType  string
	Similarity Similarity
}

var matchTypes = []string{"exact", "very_similar", "similar", "somewhat_similar", "weak"}

// FindBestMatches for each query (comparison.go:197-263).
func (g *Gallery) FindBestMatches(queries, candidates []int64, cfg CompareConfig) ([][]Match, error) {
	c := cfgOf(cfg)
	nq, nc, K := len(queries), len(candidates), cfg.MaxCandidates
	if K < 0 {
		K = 0
	}
	buf := make([]C.sonar_match, nq*K+1)
	n := make([]C.int64_t, nq+1)
	var qp, cp *C.int64_t
	if nq > 0 {
		qp = (*C.int64_t)(unsafe.Pointer(&queries[0]))
	}
	if nc > 0 {
		cp = (*C.int64_t)(unsafe.Pointer(&candidates[0]))
	}
	if rc := C.sonar_find_best_matches(g.g, qp, C.int64_t(nq), cp, C.int64_t(nc), &c, &buf[0], &n[0]); rc != 0 {
		return nil, g.x.err(rc)
	}
	out := make([][]Match, nq)
	for q := range out {
		for k := 0; k < int(n[q]); k++ {
			m := &buf[q*K+k]
			out[q] = append(out[q], Match{Candidate: candidates[int64(m.candidate)], Rank: int(m.rank),
				MatchType: matchTypes[m.match_type], Similarity: simOf(&m.similarity)})
		}
	}
	return out, nil
}

// LocalMatches is one rank's FindBestMatches output in the C ABI's layout (nq x MaxCandidates
// records, Counts[q] valid in row q): what a rank of a distributed gallery ships to the others.
type LocalMatches struct {
	Records    []C.sonar_match
	Counts     []int64
	Candidates int64 // this rank's candidate count (the next rank's numbering starts after it)
}

// FindBestMatchesLocal ranks this gallery's candidates for each query and keeps the raw lists
// for MergeMatches (the rank-local half of a FindBestMatches over several galleries).
func (g *Gallery) FindBestMatchesLocal(queries, candidates []int64, cfg CompareConfig) (*LocalMatches, error) {
	c := cfgOf(cfg)
	nq, nc, K := len(queries), len(candidates), cfg.MaxCandidates
	if K < 0 {
		K = 0
	}
	buf := make([]C.sonar_match, nq*K+1)
	n := make([]int64, nq+1)
	var qp, cp *C.int64_t
	if nq > 0 {
		qp = (*C.int64_t)(unsafe.Pointer(&queries[0]))
	}
	if nc > 0 {
		cp = (*C.int64_t)(unsafe.Pointer(&candidates[0]))
	}
	if rc := C.sonar_find_best_matches(g.g, qp, C.int64_t(nq), cp, C.int64_t(nc), &c, &buf[0],
		(*C.int64_t)(unsafe.Pointer(&n[0]))); rc != 0 {
		return nil, g.x.err(rc)
	}
	return &LocalMatches{Records: buf[:nq*K], Counts: n[:nq], Candidates: int64(nc)}, nil
}

// MergeMatches gives the FindBestMatches result of one call over the concatenated candidates of
// every rank (rank r's numbered after ranks 0..r-1): sonar_merge_matches, the single call's order.
// Candidate in the returned matches is the global position.
func MergeMatches(parts []*LocalMatches, nq, maxCandidates int) ([][]Match, error) {
	K := maxCandidates
	if K < 0 {
		K = 0
	}
	R := len(parts)
	lists := C.calloc(C.size_t(R+1), C.size_t(unsafe.Sizeof(uintptr(0))))
	defer C.free(lists)
	var pin runtime.Pinner
	defer pin.Unpin()
	counts := make([]int64, R*nq+1)
	base := make([]int64, R+1)
	for r, p := range parts {
		if len(p.Records) > 0 {
			pin.Pin(&p.Records[0])
			(*[1 << 28]unsafe.Pointer)(lists)[r] = unsafe.Pointer(&p.Records[0])
		}
		copy(counts[r*nq:], p.Counts)
		if r > 0 {
			base[r] = base[r-1] + parts[r-1].Candidates
		}
	}
	out := make([]C.sonar_match, nq*K+1)
	n := make([]int64, nq+1)
	if rc := C.sonar_merge_matches((**C.sonar_match)(lists), (*C.int64_t)(unsafe.Pointer(&counts[0])),
		(*C.int64_t)(unsafe.Pointer(&base[0])), C.int32_t(R), C.int64_t(nq), C.int32_t(K), &out[0],
		(*C.int64_t)(unsafe.Pointer(&n[0]))); rc != 0 {
		return nil, fmt.Errorf("sonar_merge_matches: %w", ErrInvalid)
	}
	res := make([][]Match, nq)
	for q := range res {
		for k := 0; k < int(n[q]); k++ {
			m := &out[q*K+k]
			res[q] = append(res[q], Match{Candidate: int64(m.candidate), Rank: int(m.rank),
				MatchType: matchTypes[m.match_type], Similarity: simOf(&m.similarity)})
		}
	}
	return res, nil
}

// FindBestMatches over rank-local galleries of one process's devices (sonar_find_best_matches_multi):
// galleries[g] must live on x's rank g; queries[g] are the queries' indices there and candidates[g]
// rank g's candidates.  The per-rank top lists travel through one RCCL all-gather.
func (x *Multi) FindBestMatches(galleries []*Gallery, queries, candidates [][]int64, cfg CompareConfig) ([][]Match,
	error) {
	G := len(galleries)
	if G == 0 || len(queries) != G || len(candidates) != G {
		return nil, fmt.Errorf("one gallery, query list and candidate list per rank: %w", ErrInvalid)
	}
	nq := len(queries[0])
	K := cfg.MaxCandidates
	if K < 0 {
		K = 0
	}
	c := cfgOf(cfg)
	ptrs := C.calloc(C.size_t(3*G), C.size_t(unsafe.Sizeof(uintptr(0))))
	defer C.free(ptrs)
	arr := (*[1 << 28]unsafe.Pointer)(ptrs)
	var pin runtime.Pinner
	defer pin.Unpin()
	nc := make([]int64, G)
	for g := 0; g < G; g++ {
		arr[g] = unsafe.Pointer(galleries[g].g)
		if len(queries[g]) > 0 {
			pin.Pin(&queries[g][0])
			arr[G+g] = unsafe.Pointer(&queries[g][0])
		}
		if len(candidates[g]) > 0 {
			pin.Pin(&candidates[g][0])
			arr[2*G+g] = unsafe.Pointer(&candidates[g][0])
		}
		nc[g] = int64(len(candidates[g]))
	}
	out := make([]C.sonar_match, nq*K+1)
	n := make([]int64, nq+1)
	if rc := C.sonar_find_best_matches_multi(x.m, (**C.sonar_gallery)(ptrs), (**C.int64_t)(unsafe.Pointer(&arr[G])),
		C.int64_t(nq), (**C.int64_t)(unsafe.Pointer(&arr[2*G])), (*C.int64_t)(unsafe.Pointer(&nc[0])), &c, &out[0],
		(*C.int64_t)(unsafe.Pointer(&n[0]))); rc != 0 {
		return nil, x.err(rc)
	}
	res := make([][]Match, nq)
	for q := range res {
		for k := 0; k < int(n[q]); k++ {
			m := &out[q*K+k]
			res[q] = append(res[q], Match{Candidate: int64(m.candidate), Rank: int(m.rank),
				MatchType: matchTypes[m.match_type], Similarity: simOf(&m.similarity)})
		}
	}
	return res, nil
}
