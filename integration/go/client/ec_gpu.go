// +build rsgpu

// ec_gpu.go — the MI355X (gfx950) erasure coder behind reedsolomon.Encoder,
// a drop-in for the encoder NewEncoder builds (client/ec.go:14-24; held in
// Client.EC, client/client.go:38; called from exactly client/ecRedis.go:384,
// 390, 395, 406, 415, 420, 430).  All GF(2^8) arithmetic runs in librsgpu.so
// (include/rsgpu.h); Split and Join stay Go host slicing with the upstream
// v1.9.3 semantics.
//
// NOT COMPILED HERE: neither this container nor the GPU box has a Go
// toolchain (profiles/r01_go_probe.txt).  Written against include/rsgpu.h and
// the reedsolomon v1.9.3 Encoder interface (go.mod:16, Go 1.12: no
// unsafe.Slice); every C entry point it calls is exercised from plain C by
// tests/c_abi_client.c (the ecredis replay) and from Python by the GPU tests.
//
// cgo pointer rules.  A call may pass a Go pointer only to Go memory that
// holds no Go pointers, and C must not keep it.  A [][]byte table holds Go
// pointers, so it never crosses.  Instead:
//   (i)  Split's output is consecutive slices of ONE backing array
//        (ecRedis.go:384).  contiguous() checks &shards[i][0] == base + i*S and
//        the *_image calls take base alone: one Go pointer to plain bytes.
//   (ii) EcGet's shards are separate buffers (ecRedis.go:161-170, 348-362).
//        They are copied into a C-owned pinned image (rsgpu_host_alloc, pooled
//        per encoder); the kernels read and write that image in place over
//        PCIe, and the rebuilt shards are copied out into Go buffers that
//        follow upstream's reuse-cap-else-allocate rule.
// librsgpu never retains a pointer past a call; every call is synchronous.
package client

/*
#cgo CFLAGS: -I${SRCDIR}/rsgpu
#cgo LDFLAGS: -L${SRCDIR}/rsgpu -lrsgpu -Wl,-rpath,${SRCDIR}/rsgpu
#include <stdlib.h>
#include "rsgpu.h"
*/
import "C"

import (
	"errors"
	"io"
	"os"
	"runtime"
	"strconv"
	"strings"
	"sync"
	"unsafe"

	"github.com/klauspost/reedsolomon"
)

type gpuEncoder struct {
	ctx          *C.rsgpu_ctx
	DataShards   int
	ParityShards int
	Shards       int
	stage        stagePool
}

// useGPU: built with -tags rsgpu, the GPU coder is the default; INFINICACHE_EC=cpu
// selects upstream's CPU coder.
func useGPU() bool { return os.Getenv("INFINICACHE_EC") != "cpu" }

// Error codes -> the upstream error VALUES, so callers' comparisons keep working.
func rsErr(code C.int) error {
	switch code {
	case C.RSGPU_OK:
		return nil
	case C.RSGPU_ERR_INV_SHARD_NUM:
		return reedsolomon.ErrInvShardNum
	case C.RSGPU_ERR_MAX_SHARD_NUM:
		return reedsolomon.ErrMaxShardNum
	case C.RSGPU_ERR_TOO_FEW_SHARDS:
		return reedsolomon.ErrTooFewShards
	case C.RSGPU_ERR_SHARD_NO_DATA:
		return reedsolomon.ErrShardNoData
	case C.RSGPU_ERR_SHARD_SIZE:
		return reedsolomon.ErrShardSize
	case C.RSGPU_ERR_SHORT_DATA:
		return reedsolomon.ErrShortData
	case C.RSGPU_ERR_RECONSTRUCT_REQUIRED:
		return reedsolomon.ErrReconstructRequired
	case C.RSGPU_ERR_INVALID_INPUT:
		return reedsolomon.ErrInvalidInput
	case C.RSGPU_ERR_NOT_IMPLEMENTED:
		return ErrNotImplemented
	default: // errSingular is unexported upstream; device/HIP failures
		return errors.New(C.GoString(C.rsgpu_strerror(code)))
	}
}

// newGPUEncoder builds the coder over every visible gfx950 GPU of this
// process (the client is one process; concurrent EcSet/EcGet calls go to the
// GPUs round-robin, one PCIe link each), or the devices listed in
// INFINICACHE_EC_DEVICES ("0,1,...").
func newGPUEncoder(dataShards, parityShards int) (reedsolomon.Encoder, error) {
	var ctx *C.rsgpu_ctx
	var rc C.int
	if list := os.Getenv("INFINICACHE_EC_DEVICES"); list != "" && list != "all" {
		fields := strings.Split(list, ",")
		devs := (*[256]C.int)(C.malloc(C.size_t(len(fields)) * C.size_t(unsafe.Sizeof(C.int(0)))))
		defer C.free(unsafe.Pointer(devs))
		for i, f := range fields {
			d, err := strconv.Atoi(strings.TrimSpace(f))
			if err != nil || i >= 256 {
				return nil, errors.New("INFINICACHE_EC_DEVICES: bad device list " + list)
			}
			devs[i] = C.int(d)
		}
		rc = C.rsgpu_create_multi(C.int(dataShards), C.int(parityShards), &devs[0], C.int(len(fields)), 0, &ctx)
	} else {
		rc = C.rsgpu_create(C.int(dataShards), C.int(parityShards), C.RSGPU_ALL_DEVICES, 0, &ctx)
	}
	if rc != 0 {
		return nil, rsErr(rc)
	}
	// No usable gfx950 device behind the context (RSGPU_ALL_DEVICES falls back
	// to a device-0 context whose compute calls all fail): report an error so
	// the patched NewEncoder keeps upstream's CPU coder (ADVICE r02).
	{
		var devs [256]C.int
		nd := int(C.rsgpu_devices(ctx, &devs[0], 256))
		usable := nd > 0
		for i := 0; i < nd && i < 256 && usable; i++ {
			usable = C.rsgpu_device_ok(devs[i]) == 1
		}
		if !usable {
			C.rsgpu_destroy(ctx)
			return nil, errors.New(C.GoString(C.rsgpu_strerror(C.RSGPU_ERR_NO_DEVICE)))
		}
	}
	// One EcSet / EcGet codes one object (ecRedis.go:96, :173): the resident
	// worker answers those calls without a kernel launch per call
	// (rsgpu_worker_start).  INFINICACHE_EC_WORKER=0 keeps the stream path;
	// codes of more than 16 shards (ErrNotImplemented) keep it too.
	if os.Getenv("INFINICACHE_EC_WORKER") != "0" {
		if rc := C.rsgpu_worker_start(ctx, 0, 0, 0); rc != 0 && rc != C.RSGPU_ERR_NOT_IMPLEMENTED {
			C.rsgpu_destroy(ctx)
			return nil, rsErr(rc)
		}
	}
	e := &gpuEncoder{ctx: ctx, DataShards: dataShards, ParityShards: parityShards,
		Shards: dataShards + parityShards}
	runtime.SetFinalizer(e, func(e *gpuEncoder) {
		e.stage.drain()
		C.rsgpu_destroy(e.ctx)
	})
	return e, nil
}

// ---- helpers ---------------------------------------------------------------

// stagePool keeps C-owned pinned images (rsgpu_host_alloc) in power-of-two
// size classes (a request of size bytes gets an image of at least size; the
// caller uses its first size bytes, and rsgpu_host_alloc's 64 B of slack lie
// past the class).  Go copies shard bytes into them (C memory holding no
// pointers); the kernels access them in place.  At most 8 images per class
// and stagePoolCap bytes in all are kept: config 5 mixes 4 KiB-100 MiB
// objects, and an exact-size pool kept one set per distinct size.  Each
// rsgpu_host_free parks a resident worker for its duration (rsgpu.h), so the
// pool frees rarely.
type stagePool struct {
	mu    sync.Mutex
	free  map[int][]unsafe.Pointer
	bytes int
}

const stagePoolCap = 512 << 20

func stageClass(size int) int {
	c := 4096
	for c < size {
		c <<= 1
	}
	return c
}

func (p *stagePool) get(size int) (unsafe.Pointer, error) {
	cls := stageClass(size)
	p.mu.Lock()
	if l := p.free[cls]; len(l) > 0 {
		ptr := l[len(l)-1]
		p.free[cls] = l[:len(l)-1]
		p.bytes -= cls
		p.mu.Unlock()
		return ptr, nil
	}
	p.mu.Unlock()
	var ptr unsafe.Pointer
	if rc := C.rsgpu_host_alloc(C.size_t(cls), &ptr); rc != 0 {
		return nil, rsErr(rc)
	}
	return ptr, nil
}

func (p *stagePool) put(size int, ptr unsafe.Pointer) {
	cls := stageClass(size)
	p.mu.Lock()
	if p.free == nil {
		p.free = map[int][]unsafe.Pointer{}
	}
	if len(p.free[cls]) < 8 && p.bytes+cls <= stagePoolCap {
		p.free[cls] = append(p.free[cls], ptr)
		p.bytes += cls
		ptr = nil
	}
	p.mu.Unlock()
	if ptr != nil {
		C.rsgpu_host_free(ptr)
	}
}

func (p *stagePool) drain() {
	p.mu.Lock()
	defer p.mu.Unlock()
	for _, l := range p.free {
		for _, ptr := range l {
			C.rsgpu_host_free(ptr)
		}
	}
	p.free = nil
	p.bytes = 0
}

// cbytes is a Go view of n bytes of C memory (Go 1.12: no unsafe.Slice).
func cbytes(p unsafe.Pointer, n int) []byte { return (*[1 << 40]byte)(p)[:n:n] }

// contiguous: Split's layout, every shard S > 0 bytes at base + i*S.
func contiguous(shards [][]byte) (*byte, int, bool) {
	if len(shards) == 0 || len(shards[0]) == 0 {
		return nil, 0, false
	}
	S := len(shards[0])
	base := uintptr(unsafe.Pointer(&shards[0][0]))
	for i, s := range shards {
		if len(s) != S || uintptr(unsafe.Pointer(&s[0])) != base+uintptr(i*S) {
			return nil, 0, false
		}
	}
	return &shards[0][0], S, true
}

// checkShards: upstream's (size = first non-empty length; ErrShardNoData /
// ErrShardSize), so staged calls keep the same error precedence.
func checkShards(shards [][]byte, nilok bool) (int, error) {
	size := 0
	for _, s := range shards {
		if len(s) != 0 {
			size = len(s)
			break
		}
	}
	if size == 0 {
		return 0, reedsolomon.ErrShardNoData
	}
	for _, s := range shards {
		if len(s) != size && (len(s) != 0 || !nilok) {
			return 0, reedsolomon.ErrShardSize
		}
	}
	return size, nil
}

func u8(p unsafe.Pointer) *C.uint8_t { return (*C.uint8_t)(p) }

// ---- reedsolomon.Encoder ------------------------------------------------------

func (e *gpuEncoder) Encode(shards [][]byte) error {
	if len(shards) != e.Shards {
		return reedsolomon.ErrTooFewShards
	}
	if base, S, ok := contiguous(shards); ok { // route (i)
		rc := C.rsgpu_encode_image(e.ctx, (*C.uint8_t)(unsafe.Pointer(base)), C.size_t(S), C.int(e.Shards))
		runtime.KeepAlive(shards)
		return rsErr(rc)
	}
	S, err := checkShards(shards, false)
	if err != nil {
		return err
	}
	return e.staged(shards, S, func(img unsafe.Pointer) C.int { // route (ii)
		return C.rsgpu_encode_image(e.ctx, u8(img), C.size_t(S), C.int(e.Shards))
	}, e.DataShards, e.Shards)
}

// staged copies rows [0, in) into a pooled C image, runs f on it, and copies
// rows [in, out) back into shards.
func (e *gpuEncoder) staged(shards [][]byte, S int, f func(unsafe.Pointer) C.int, in, out int) error {
	size := e.Shards * S
	img, err := e.stage.get(size)
	if err != nil {
		return err
	}
	defer e.stage.put(size, img)
	view := cbytes(img, size)
	for i := 0; i < in; i++ {
		copy(view[i*S:(i+1)*S], shards[i])
	}
	if rc := f(img); rc != 0 {
		return rsErr(rc)
	}
	for i := in; i < out; i++ {
		copy(shards[i], view[i*S:(i+1)*S])
	}
	return nil
}

// Client.decode calls Verify on Get results that always hold nil shards
// (proxy first-d rule).  Upstream answers (false, ErrShardSize) without any
// math; so does this, before any cgo call.
func (e *gpuEncoder) Verify(shards [][]byte) (bool, error) {
	if len(shards) != e.Shards {
		return false, reedsolomon.ErrTooFewShards
	}
	S, err := checkShards(shards, false)
	if err != nil {
		return false, err
	}
	var ok C.int
	if base, _, c := contiguous(shards); c {
		rc := C.rsgpu_verify_image(e.ctx, (*C.uint8_t)(unsafe.Pointer(base)), C.size_t(S), C.int(e.Shards), &ok)
		runtime.KeepAlive(shards)
		return ok != 0, rsErr(rc)
	}
	err = e.staged(shards, S, func(img unsafe.Pointer) C.int {
		return C.rsgpu_verify_image(e.ctx, u8(img), C.size_t(S), C.int(e.Shards), &ok)
	}, e.Shards, e.Shards)
	return ok != 0, err
}

// EncodeVerify: Client.encode's Encode -> Verify pair (ecRedis.go:390-395) in
// one device round trip; returns exactly what the Verify would (fusedCoder).
func (e *gpuEncoder) EncodeVerify(shards [][]byte) (bool, error) {
	if len(shards) != e.Shards {
		return false, reedsolomon.ErrTooFewShards
	}
	var ok C.int
	if base, S, c := contiguous(shards); c {
		rc := C.rsgpu_encode_verify_image(e.ctx, (*C.uint8_t)(unsafe.Pointer(base)), C.size_t(S),
			C.int(e.Shards), &ok)
		runtime.KeepAlive(shards)
		return ok != 0, rsErr(rc)
	}
	S, err := checkShards(shards, false)
	if err != nil {
		return false, err
	}
	err = e.staged(shards, S, func(img unsafe.Pointer) C.int {
		return C.rsgpu_encode_verify_image(e.ctx, u8(img), C.size_t(S), C.int(e.Shards), &ok)
	}, e.DataShards, e.Shards)
	return ok != 0, err
}

func (e *gpuEncoder) Reconstruct(shards [][]byte) error {
	_, err := e.reconstruct(shards, false, false)
	return err
}

func (e *gpuEncoder) ReconstructData(shards [][]byte) error {
	_, err := e.reconstruct(shards, true, false)
	return err
}

// DecodeVerify: Client.decode's Reconstruct -> Verify pair (ecRedis.go:415-420)
// in one device pass (rsgpu_decode_image); returns what that Verify would.
func (e *gpuEncoder) DecodeVerify(shards [][]byte) (bool, error) {
	return e.reconstruct(shards, false, true)
}

// reconstruct: route (ii).  The present shards go into a pooled C image, the
// device rebuilds the missing ones in place, and each missing shard i gets a
// Go buffer as upstream gives it (shards[i][:size] when cap allows, else a new
// slice) holding the rebuilt bytes.
func (e *gpuEncoder) reconstruct(shards [][]byte, dataOnly, verify bool) (bool, error) {
	if len(shards) != e.Shards {
		return false, reedsolomon.ErrTooFewShards
	}
	S, err := checkShards(shards, true)
	if err != nil {
		return false, err
	}
	var present C.uint64_t
	np := 0
	for i, s := range shards {
		if len(s) != 0 {
			present |= 1 << uint(i)
			np++
		}
	}
	if np == e.Shards && !verify {
		return true, nil // upstream: nothing to do
	}
	if np < e.DataShards {
		return false, reedsolomon.ErrTooFewShards
	}
	if e.Shards > 64 {
		return false, ErrNotImplemented // image calls carry a 64-bit present mask
	}
	size := e.Shards * S
	img, err := e.stage.get(size)
	if err != nil {
		return false, err
	}
	defer e.stage.put(size, img)
	view := cbytes(img, size)
	for i, s := range shards {
		if len(s) != 0 {
			copy(view[i*S:(i+1)*S], s)
		}
	}
	var ok C.int
	var rc C.int
	if verify {
		rc = C.rsgpu_decode_image(e.ctx, u8(img), C.size_t(S), C.int(e.Shards), present, &ok)
	} else {
		rc = C.rsgpu_reconstruct_image(e.ctx, u8(img), C.size_t(S), C.int(e.Shards), present, cbool(dataOnly))
	}
	if rc != 0 {
		return false, rsErr(rc)
	}
	for i := range shards {
		if len(shards[i]) != 0 || (dataOnly && i >= e.DataShards) {
			continue
		}
		if cap(shards[i]) >= S {
			shards[i] = shards[i][0:S]
		} else {
			shards[i] = make([]byte, S)
		}
		copy(shards[i], view[i*S:(i+1)*S])
	}
	return ok != 0, nil
}

// Update: upstream semantics (shards[c] for each non-nil newDatashards[c]
// becomes the delta old^new, parity is updated by M[.,c] x delta).  All rows
// are staged; the C-side pointer tables live in C memory.
func (e *gpuEncoder) Update(shards [][]byte, newDatashards [][]byte) error {
	if len(shards) != e.Shards || len(newDatashards) != e.DataShards {
		return reedsolomon.ErrTooFewShards
	}
	S, err := checkShards(shards, true)
	if err != nil {
		return err
	}
	if _, err := checkShards(newDatashards, true); err != nil {
		return err
	}
	n, k := e.Shards, e.DataShards
	size := (n + k) * S
	img, err := e.stage.get(size)
	if err != nil {
		return err
	}
	defer e.stage.put(size, img)
	view := cbytes(img, size)
	ptrs := (*[512]*C.uint8_t)(C.malloc(C.size_t(n+k) * C.size_t(unsafe.Sizeof(uintptr(0)))))
	lens := (*[512]C.size_t)(C.malloc(C.size_t(n+k) * C.size_t(unsafe.Sizeof(C.size_t(0)))))
	defer C.free(unsafe.Pointer(ptrs))
	defer C.free(unsafe.Pointer(lens))
	rows := append(append([][]byte{}, shards...), newDatashards...)
	for i, s := range rows {
		ptrs[i] = u8(unsafe.Pointer(&view[i*S]))
		lens[i] = C.size_t(len(s))
		copy(view[i*S:(i+1)*S], s)
	}
	rc := C.rsgpu_update(e.ctx, &ptrs[0], &lens[0], C.int(n), &ptrs[n], &lens[n], C.int(k))
	if rc != 0 {
		return rsErr(rc)
	}
	for i := 0; i < n; i++ {
		if len(shards[i]) != 0 {
			copy(shards[i], view[i*S:(i+1)*S])
		}
	}
	return nil
}

// Split / Join: upstream v1.9.3 semantics (pure host slicing).
func (e *gpuEncoder) Split(data []byte) ([][]byte, error) {
	if len(data) == 0 {
		return nil, reedsolomon.ErrShortData
	}
	perShard := (len(data) + e.DataShards - 1) / e.DataShards
	if cap(data) > len(data) {
		data = data[:cap(data)]
	}
	if len(data) < e.Shards*perShard {
		data = append(data, make([]byte, e.Shards*perShard-len(data))...)
	}
	dst := make([][]byte, e.Shards)
	for i := range dst {
		dst[i] = data[:perShard]
		data = data[perShard:]
	}
	return dst, nil
}

func (e *gpuEncoder) Join(dst io.Writer, shards [][]byte, outSize int) error {
	return (&DummyEncoder{DataShards: e.DataShards}).Join(dst, shards, outSize) // same logic, ec.go:83-121
}

func cbool(b bool) C.int {
	if b {
		return 1
	}
	return 0
}
