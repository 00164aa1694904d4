// fused.go — optional one-round-trip forms of Client.encode's Encode->Verify
// pair (ecRedis.go:390-395) and Client.decode's Reconstruct->Verify pair
// (ecRedis.go:415-420).  The GPU coder implements fusedCoder; upstream's CPU
// coder does not, so Client.encode/decode keep their exact flow unless the
// maintainer adds the assertion shown in ecRedis.go.patch.
// NOT COMPILED HERE (no Go toolchain; see ec_gpu.go).
package client

type fusedCoder interface {
	EncodeVerify(shards [][]byte) (bool, error)
	DecodeVerify(shards [][]byte) (bool, error)
}
