// Parity of the cgo binding against the reference's own bitcoin.Hash
// (src/github.com/cmu440/bitcoin/hash.go:11-15): the test a maintainer runs on a GPU
// box that has Go (SURVEY.md 8(f) row 1, "a Go test comparing it to bitcoin.Hash").
//
// NOT COMPILED IN THIS REPO: there is no Go toolchain in the build container or on the
// GPU box (INTEGRATION.md).  The same checks run there against the C and hashlib
// restatements of hash.go (tests/test_gpu.py); tests/test_abi.py checks that every C
// identifier used here and in gpuhash.go is declared in include/gpuhash.h.
//
//	CGO_CFLAGS="-I<repo>/include" CGO_LDFLAGS="-L<repo>/bitcoin-miner_amd/lib" go test ./...
package gpuhash

import (
	"math"
	"testing"

	"github.com/cmu440/bitcoin"
)

// the spec'd miner loop (p1.pdf pp.12-14): ascending, strict '<', lowest nonce on ties
func scan(msg string, lower, upper uint64) (uint64, uint64) {
	best, bn := bitcoin.Hash(msg, lower), lower
	for n := lower; n != upper; {
		n++
		if h := bitcoin.Hash(msg, n); h < best {
			best, bn = h, n
		}
	}
	return best, bn
}

func open(t *testing.T) *Engine {
	e, err := Open()
	if err != nil {
		t.Skipf("no MI355X: %v", err)
	}
	return e
}

func TestHandoutValues(t *testing.T) {
	e := open(t)
	defer e.Close()
	// p1.pdf p.12
	h, n, err := e.Min("msg", 0, 2)
	if err != nil || h != 4754799531757243342 || n != 1 {
		t.Fatalf("Min(msg, 0, 2) = %d %d %v", h, n, err)
	}
	// BASELINE config 1: the client must print "Result 1419516646206828 9898"
	h, n, err = e.Min("bradfitz", 0, 9999)
	if err != nil || h != 1419516646206828 || n != 9898 {
		t.Fatalf("Min(bradfitz, 0, 9999) = %d %d %v", h, n, err)
	}
}

func TestAgainstBitcoinHash(t *testing.T) {
	e := open(t)
	defer e.Close()
	m120 := "The quick brown fox jumps over the lazy dog. The quick brown fox jumps over the lazy dog. The quick brown fox jumps over"
	cases := []struct {
		msg          string
		lower, upper uint64
	}{
		{"", 0, 9},
		{"bradfitz", 999999000, 1000001000},           // 9 -> 10 digits
		{m120[:44], 9999999000, 10000001000},          // 10 -> 11 digits, 1 -> 2 blocks
		{m120[:45], 999999000, 1000001000},            // extra padding block
		{m120, 9999999000, 10000001000},               // config 3's boundary
		{"bradfitz", math.MaxUint64 - 3000, math.MaxUint64}, // 20 digits, no overflow
		{"héllo ✓", 123456789, 123556789},             // Data is hashed as its UTF-8 bytes
	}
	for _, c := range cases {
		h, n, err := e.Min(c.msg, c.lower, c.upper)
		if err != nil {
			t.Fatalf("%q [%d, %d]: %v", c.msg, c.lower, c.upper, err)
		}
		wh, wn := scan(c.msg, c.lower, c.upper)
		if h != wh || n != wn {
			t.Fatalf("%q [%d, %d]: gpu (%d, %d), bitcoin.Hash loop (%d, %d)", c.msg, c.lower, c.upper, h, n, wh, wn)
		}
	}
}

func TestErrorClasses(t *testing.T) {
	e := open(t)
	defer e.Close()
	_, _, err := e.Min("x", 10, 9) // lower > upper
	ge, ok := err.(*Error)
	if !ok || !ge.IsArgument() {
		t.Fatalf("lower > upper: %v, want an argument error", err)
	}
}
