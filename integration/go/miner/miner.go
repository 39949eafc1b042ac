// The reference miner (src/github.com/cmu440/bitcoin/miner/miner.go, a stub whose
// body is "// TODO: implement this!" at :15) written the way the handout specifies it
// (p1.pdf pp.13-15), with the min-hash loop replaced by one gpuhash call.  Only the
// loop changes; Join / Read / Write / exit-on-lost-server are the reference's protocol.
//
// NOT COMPILED IN THIS REPO (no Go toolchain here or on the GPU box); see
// INTEGRATION.md.  Note the reference LSP client cannot carry data as written
// (SURVEY.md 2, rows 8-9), so running this end to end also needs a working lsp/.
package main

import (
	"encoding/json"
	"errors"
	"fmt"
	"log"
	"math"
	"os"

	"github.com/cmu440/bitcoin"
	"github.com/cmu440/gpuhash"
	"github.com/cmu440/lsp"
)

func main() {
	const numArgs = 2
	if len(os.Args) != numArgs {
		fmt.Println("Usage: ./miner <hostport>")
		return
	}
	client, err := lsp.NewClient(os.Args[1], lsp.NewParams())
	if err != nil {
		return
	}
	defer client.Close()
	eng, err := gpuhash.Open() // all visible MI355X GPUs (HIP_VISIBLE_DEVICES narrows it)
	if err != nil {
		return
	}
	defer eng.Close()
	join, _ := json.Marshal(bitcoin.NewJoin())
	if client.Write(join) != nil {
		return
	}
	for {
		payload, err := client.Read()
		if err != nil {
			return // server lost (p1.pdf p.15)
		}
		var req bitcoin.Message
		if json.Unmarshal(payload, &req) != nil || req.Type != bitcoin.Request {
			continue
		}
		if req.Lower > req.Upper {
			// the spec'd loop runs zero times: reply with the min over the empty set, the
			// top of the (hash, nonce) order, which the server's merge ignores
			res, _ := json.Marshal(bitcoin.NewResult(math.MaxUint64, math.MaxUint64))
			if client.Write(res) != nil {
				return
			}
			continue
		}
		// was: for n := req.Lower; n <= req.Upper; n++ { h := bitcoin.Hash(req.Data, n) ... }
		hash, nonce, err := eng.Min(req.Data, req.Lower, req.Upper)
		if err != nil {
			// Argument errors (ge.IsArgument) as much as device errors: no Result can be
			// sent, and skipping the job would leave it in flight forever (the server
			// pairs each Result with the miner's oldest job).  Exiting drops the
			// connection, the server requeues the job (p1.pdf p.15), and its requeue cap
			// disconnects the client if every miner fails it the same way.
			var ge *gpuhash.Error
			log.Printf("miner: job %v failed (argument error: %v): %v; exiting", req, errors.As(err, &ge) && ge.IsArgument(), err)
			return
		}
		// optional self-check against the unmodified reference hash
		if bitcoin.Hash(req.Data, nonce) != hash {
			return
		}
		res, _ := json.Marshal(bitcoin.NewResult(hash, nonce))
		if client.Write(res) != nil {
			return
		}
	}
}
