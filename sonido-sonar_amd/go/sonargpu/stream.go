package sonargpu

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

// SpectrogramFrame mirrors analyzers.SpectrogramFrame (fingerprint/analyzers/spectral.go:369-374).
type SpectrogramFrame struct {
	Magnitude []float64
	Phase     []float64
	Complex   []complex128
}

// STFTStreamer is analyzers.STFTStreamer (spectral.go:314-321) with Go's buffer kept on the GPU:
// each ProcessChunk appends the chunk behind the unconsumed samples and emits every complete frame
// in one fused launch.  Like the Go streamer it is not goroutine-safe; it shares its Context's
// HIP stream.
type STFTStreamer struct {
	x         *Context
	st        *C.sonar_stft_stream
	freqBins  int
	windowLen int
}

// ComputeSTFTStreaming is SpectralAnalyzer.ComputeSTFTStreaming (spectral.go:289-312) on the GPU,
// float64 ({Normalize, Symmetric} window, Beta / Alpha at Go's zero value as in the reference).
func (x *Context) ComputeSTFTStreaming(windowSize, hopSize, windowType int) (*STFTStreamer, error) {
	var cfg C.sonar_fp_cfg
	C.sonar_fp_cfg_default(&cfg)
	cfg.window_size, cfg.hop_size, cfg.window_type = C.int32_t(windowSize), C.int32_t(hopSize), C.int32_t(windowType)
	cfg.flags = C.SONAR_FP_MAGNITUDE | C.SONAR_FP_PHASE | C.SONAR_FP_COMPLEX
	cfg.precision, cfg.pcm_dtype, cfg.out_dtype = C.SONAR_F64, C.SONAR_F64, C.SONAR_F64
	var st *C.sonar_stft_stream
	if rc := C.sonar_stft_stream_create(x.c, &cfg, &st); rc != C.SONAR_OK {
		return nil, x.err(rc)
	}
	return &STFTStreamer{x: x, st: st, freqBins: windowSize/2 + 1, windowLen: windowSize}, nil
}

// ProcessChunk is STFTStreamer.ProcessChunk (spectral.go:322-366): nil, nil for an empty chunk.
// A zero hop returns an error where Go's loop would not terminate; a negative one ErrPanic with
// Go's slice-bounds message.
func (s *STFTStreamer) ProcessChunk(chunk []float64) ([]*SpectrogramFrame, error) {
	if len(chunk) == 0 {
		return nil, nil
	}
	n := C.int64_t(len(chunk))
	frames := int(C.sonar_stft_stream_frames(s.st, n))
	if frames < 0 {
		frames = 0 // the push reports the error
	}
	k := s.freqBins
	// The output struct holds pointers to Go memory: cgo's pointer check rejects a Go pointer to
	// unpinned Go pointers, so the row slices (and the chunk) are pinned for the call.
	var pin runtime.Pinner
	defer pin.Unpin()
	out := (*C.sonar_fp_out)(C.calloc(1, C.size_t(unsafe.Sizeof(C.sonar_fp_out{}))))
	defer C.free(unsafe.Pointer(out))
	var mag, ph []float64
	var cx []complex128
	if frames > 0 {
		mag, ph, cx = make([]float64, frames*k), make([]float64, frames*k), make([]complex128, frames*k)
		pin.Pin(&mag[0])
		pin.Pin(&ph[0])
		pin.Pin(&cx[0])
		out.magnitude, out.phase, out.complex = unsafe.Pointer(&mag[0]), unsafe.Pointer(&ph[0]), unsafe.Pointer(&cx[0])
	}
	pin.Pin(&chunk[0])
	var got C.int64_t
	if rc := C.sonar_stft_stream_push(s.st, unsafe.Pointer(&chunk[0]), n, out, &got); rc != C.SONAR_OK {
		return nil, s.x.err(rc)
	}
	if int(got) != frames {
		return nil, fmt.Errorf("sonargpu: stream emitted %d frames, expected %d: %w", int(got), frames, ErrDevice)
	}
	if frames == 0 {
		return nil, nil // Go's ProcessChunk returns a nil slice when no frame completes (spectral.go:331, 373)
	}
	res := make([]*SpectrogramFrame, frames)
	for t := range res {
		res[t] = &SpectrogramFrame{Magnitude: mag[t*k : (t+1)*k], Phase: ph[t*k : (t+1)*k],
			Complex: cx[t*k : (t+1)*k]}
	}
	return res, nil
}

// Buffered is len(s.buffer) of the Go streamer: samples waiting for the next frame.
func (s *STFTStreamer) Buffered() int { return int(C.sonar_stft_stream_buffered(s.st)) }

// Close releases the device buffers (the Go streamer needs no Close; call it when done).
func (s *STFTStreamer) Close() {
	if s.st != nil {
		C.sonar_stft_stream_destroy(s.st)
		s.st = nil
	}
}
