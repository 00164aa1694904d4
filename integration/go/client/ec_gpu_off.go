// +build !rsgpu

// ec_gpu_off.go — without -tags rsgpu the client keeps upstream's CPU coder:
// NewEncoder (client/ec.go, patched by ec.go.patch) never takes the GPU branch.
// NOT COMPILED HERE (no Go toolchain; see ec_gpu.go).
package client

import (
	"errors"

	"github.com/klauspost/reedsolomon"
)

func useGPU() bool { return false }

func newGPUEncoder(dataShards, parityShards int) (reedsolomon.Encoder, error) {
	return nil, errors.New("rsgpu: client built without -tags rsgpu")
}
