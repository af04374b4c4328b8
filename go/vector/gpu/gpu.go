//go:build linux && cgo

// Package gpu serves Weaviate's VectorIndex search path from libwvgpu.so, the
// MI355X engine of this repository, behind the reference's own interface
// (adapters/repos/db/vector_index.go:23-40).  It is the file a maintainer
// commits as adapters/repos/db/vector/gpu/gpu.go; the one-line factory change
// in adapters/repos/db/shard.go:134-172 is shown in INTEGRATION.md.
//
// The decorator owns a GPU mirror of one shard's hnsw index and delegates
// persistence (commit log, snapshots), maintenance and every write to the CPU
// index it wraps, then propagates the write to the mirror:
//
//	Add(id, vec)     -> cpu.Add, then wv_index_add            (insert.go:43-65)
//	Delete(ids...)   -> cpu.Delete, then wv_index_add_tombstones (delete.go:29-84)
//	SearchByVector   -> wv_batcher_search (concurrent callers coalesced into
//	                    one GPU batch; search.go:64-79 dispatch inside)
//	SearchByVectorDistance -> wv_search_by_vector_distance   (search.go:90-158)
//	UpdateUserConfig -> cpu.UpdateUserConfig, then wv_index_update_config
//
// A write the mirror cannot take (an id beyond its capacity, a device error)
// marks the mirror stale: searches are then answered by the CPU index until
// SyncFromCPU uploads a fresh snapshot, so a stale mirror never serves a
// deleted id or misses an added one.
//
// The Go toolchain is not part of the build image this engine is developed
// in; tests/native/go_replay.cpp replays this file's C call sequence
// (concurrent searches while adding and deleting) against the library on the
// GPU and asserts both properties.
package gpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../../include
#cgo LDFLAGS: -L${SRCDIR}/../../../weaviate_amd -lwvgpu -Wl,-rpath,${SRCDIR}/../../../weaviate_amd
#include <stdlib.h>
#include "wvgpu.h"
*/
import "C"

import (
	"context"
	"sync"
	"sync/atomic"
	"unsafe"

	"github.com/pkg/errors"
	"github.com/weaviate/weaviate/adapters/repos/db/helpers"
	"github.com/weaviate/weaviate/entities/schema"
	ent "github.com/weaviate/weaviate/entities/vectorindex/hnsw"
)

// cpuIndex is the VectorIndex the decorator wraps (vector_index.go:23-40).
type cpuIndex interface {
	Dump(labels ...string)
	Add(id uint64, vector []float32) error
	Delete(id ...uint64) error
	SearchByVector(vector []float32, k int, allow helpers.AllowList) ([]uint64, []float32, error)
	SearchByVectorDistance(vector []float32, dist float32, maxLimit int64,
		allow helpers.AllowList) ([]uint64, []float32, error)
	UpdateUserConfig(updated schema.VectorIndexConfig, callback func()) error
	Drop(ctx context.Context) error
	Shutdown(ctx context.Context) error
	Flush() error
	PauseMaintenance(ctx context.Context) error
	SwitchCommitLogs(ctx context.Context) error
	ListFiles(ctx context.Context) ([]string, error)
	ResumeMaintenance(ctx context.Context) error
	PostStartup()
	ValidateBeforeInsert(vector []float32) error
}

// Metric values of wv_metric (distancer.Provider.Type(), provider.go:14-24).
const (
	MetricL2Squared = C.WV_L2_SQUARED
	MetricDot       = C.WV_DOT
	MetricCosineDot = C.WV_COSINE_DOT
)

// Index is a VectorIndex whose searches run on one MI355X.
type Index struct {
	cpuIndex
	ix       *C.wv_index
	b        *C.wv_batcher
	dim      int
	capacity uint64
	device   int

	// mu: searches and propagated writes hold it shared, SyncFromCPU and
	// Shutdown exclusively (the ABI forbids uploads racing searches).
	mu    sync.RWMutex
	stale atomic.Bool
}

// Options sizes the mirror and its micro-batcher.
type Options struct {
	Device      int
	Capacity    uint64 // local ids 0..Capacity-1 (docIDs are dense per shard)
	MaxBatch    int    // queries per coalesced launch (default 1024)
	MaxWaitUsec int    // batching window after the first waiting query (default 200)
}

func lastErr(op string, rc C.int) error {
	return errors.Errorf("wvgpu %s: status %d: %s", op, int(rc), C.GoString(C.wv_last_error()))
}

func configOf(uc ent.UserConfig, device int) C.wv_config {
	var cfg C.wv_config
	C.wv_config_default(&cfg)
	cfg.device = C.int(device)
	cfg.max_connections = C.int(uc.MaxConnections)
	cfg.ef = C.int64_t(uc.EF)
	cfg.dynamic_ef_min = C.int64_t(uc.DynamicEFMin)
	cfg.dynamic_ef_max = C.int64_t(uc.DynamicEFMax)
	cfg.dynamic_ef_factor = C.int64_t(uc.DynamicEFFactor)
	cfg.flat_search_cutoff = C.int64_t(uc.FlatSearchCutoff)
	return cfg
}

// New creates the mirror; it serves searches once SyncFromCPU has uploaded
// the CPU index's state (PostStartup).
func New(cpu cpuIndex, dim int, metric int, uc ent.UserConfig, opt Options) (*Index, error) {
	if opt.MaxBatch <= 0 {
		opt.MaxBatch = 1024
	}
	if opt.MaxWaitUsec <= 0 {
		opt.MaxWaitUsec = 200
	}
	cfg := configOf(uc, opt.Device)
	var ix *C.wv_index
	if rc := C.wv_index_create(C.int(dim), C.int(metric), &cfg, C.uint64_t(opt.Capacity), &ix); rc != 0 {
		return nil, lastErr("create", rc)
	}
	var b *C.wv_batcher
	if rc := C.wv_batcher_create(ix, C.int(dim), C.int(opt.MaxBatch), C.int(opt.MaxWaitUsec), &b); rc != 0 {
		C.wv_index_destroy(ix)
		return nil, lastErr("batcher", rc)
	}
	g := &Index{cpuIndex: cpu, ix: ix, b: b, dim: dim, capacity: opt.Capacity, device: opt.Device}
	g.stale.Store(true)
	return g, nil
}

// allowBits turns the sroar-backed AllowList (helpers/allow_list.go:19-118)
// into the dense bitmap of the ABI: bit i of word i/64 <=> docID i allowed.
func allowBits(allow helpers.AllowList) ([]uint64, uint64) {
	if allow == nil {
		return nil, 0
	}
	ids := allow.Slice() // ascending
	var nbits uint64
	if len(ids) > 0 {
		nbits = ids[len(ids)-1] + 1
	}
	bits := make([]uint64, nbits/64+1)
	for _, id := range ids {
		bits[id>>6] |= 1 << (id & 63)
	}
	return bits, nbits
}

func (g *Index) markStale() {
	g.stale.Store(true)
}

// Add mirrors hnsw.Add (insert.go:43-65): the CPU index persists the node,
// then the row joins the GPU mirror (its delta set until the next snapshot),
// findable by the next search.
func (g *Index) Add(id uint64, vector []float32) error {
	if err := g.cpuIndex.Add(id, vector); err != nil {
		return err
	}
	g.mu.RLock()
	defer g.mu.RUnlock()
	if g.stale.Load() {
		return nil
	}
	if id >= g.capacity || len(vector) != g.dim {
		g.markStale() // grows past the mirror: serve from the CPU until a resync
		return nil
	}
	ids := [1]uint64{id}
	if rc := C.wv_index_add(g.ix, (*C.uint64_t)(unsafe.Pointer(&ids[0])),
		(*C.float)(unsafe.Pointer(&vector[0])), 1); rc != 0 {
		g.markStale()
	}
	return nil
}

// Delete mirrors hnsw.Delete (delete.go:29-84): tombstones, applied to the
// mirror before Delete returns, so no later search returns the ids.
func (g *Index) Delete(ids ...uint64) error {
	if err := g.cpuIndex.Delete(ids...); err != nil {
		return err
	}
	if len(ids) == 0 {
		return nil
	}
	g.mu.RLock()
	defer g.mu.RUnlock()
	if g.stale.Load() {
		return nil
	}
	in := make([]uint64, 0, len(ids))
	for _, id := range ids {
		if id < g.capacity {
			in = append(in, id)
		}
	}
	if len(in) == 0 {
		return nil
	}
	if rc := C.wv_index_add_tombstones(g.ix, (*C.uint64_t)(unsafe.Pointer(&in[0])), C.uint64_t(len(in))); rc != 0 {
		g.markStale()
	}
	return nil
}

// SearchByVector replaces hnsw.SearchByVector (search.go:64-79).  Concurrent
// callers are coalesced by the library's micro-batcher into one launch.
func (g *Index) SearchByVector(vector []float32, k int, allow helpers.AllowList) ([]uint64, []float32, error) {
	g.mu.RLock()
	if g.stale.Load() || len(vector) != g.dim || k <= 0 {
		g.mu.RUnlock()
		return g.cpuIndex.SearchByVector(vector, k, allow)
	}
	bits, nbits := allowBits(allow)
	ids := make([]uint64, k)
	dists := make([]float32, k)
	var n C.int32_t
	var bp *C.uint64_t
	if bits != nil {
		bp = (*C.uint64_t)(unsafe.Pointer(&bits[0]))
	}
	rc := C.wv_batcher_search(g.b, (*C.float)(unsafe.Pointer(&vector[0])), C.int(k), bp, C.uint64_t(nbits),
		(*C.uint64_t)(unsafe.Pointer(&ids[0])), (*C.float)(unsafe.Pointer(&dists[0])), &n)
	g.mu.RUnlock()
	if rc == C.WV_EDELETED {
		return nil, nil, errors.New("entrypoint was deleted in the object store, " +
			"it has been flagged for cleanup and should be fixed in the next cleanup cycle")
	}
	if rc != 0 {
		// device error: this call is answered by the CPU index (SURVEY §5)
		return g.cpuIndex.SearchByVector(vector, k, allow)
	}
	if n == 0 {
		return nil, nil, nil // empty index: search.go:463-465
	}
	return ids[:n], dists[:n], nil
}

// SearchByVectorDistance replaces hnsw.SearchByVectorDistance (search.go:90-158).
func (g *Index) SearchByVectorDistance(vector []float32, dist float32, maxLimit int64,
	allow helpers.AllowList) ([]uint64, []float32, error) {
	g.mu.RLock()
	defer g.mu.RUnlock()
	if g.stale.Load() || len(vector) != g.dim {
		return g.cpuIndex.SearchByVectorDistance(vector, dist, maxLimit, allow)
	}
	bits, nbits := allowBits(allow)
	var bp *C.uint64_t
	if bits != nil {
		bp = (*C.uint64_t)(unsafe.Pointer(&bits[0]))
	}
	capOut := int64(1 << 12)
	if maxLimit > 0 && maxLimit < capOut {
		capOut = maxLimit
	}
	for {
		ids := make([]uint64, capOut)
		dists := make([]float32, capOut)
		var n C.int64_t
		rc := C.wv_search_by_vector_distance(g.ix, (*C.float)(unsafe.Pointer(&vector[0])), C.float(dist),
			C.int64_t(maxLimit), bp, C.uint64_t(nbits), (*C.uint64_t)(unsafe.Pointer(&ids[0])),
			(*C.float)(unsafe.Pointer(&dists[0])), C.int64_t(capOut), &n)
		if rc != 0 {
			return g.cpuIndex.SearchByVectorDistance(vector, dist, maxLimit, allow)
		}
		if int64(n) <= capOut {
			return ids[:n], dists[:n], nil
		}
		capOut = int64(n) // the full count is known: one more call with room for it
	}
}

// UpdateUserConfig mirrors hnsw.UpdateUserConfig (config_update.go:79-120): ef,
// dynamic ef and flatSearchCutoff change the search path.
func (g *Index) UpdateUserConfig(updated schema.VectorIndexConfig, callback func()) error {
	if err := g.cpuIndex.UpdateUserConfig(updated, callback); err != nil {
		return err
	}
	uc, ok := updated.(ent.UserConfig)
	if !ok {
		return nil
	}
	g.mu.Lock()
	defer g.mu.Unlock()
	cfg := configOf(uc, g.device)
	if rc := C.wv_index_update_config(g.ix, &cfg); rc != 0 {
		g.markStale()
	}
	return nil
}

// Snapshot is the CPU index's state in the ABI's CSR layout
// (wv_index_upload_graph in include/wvgpu.h; wv_graph_export_csr builds it
// from the commit log).
type Snapshot struct {
	Vectors    []float32 // [N][dim]
	N          uint64
	Levels     []int8   // [N], -1 nil
	Layer0     []uint32 // [N][Deg0]
	Deg0       int
	UpperRow   []uint32 // [N]
	Upper      []uint32 // [NUpper][MaxLevel][DegU]
	NUpper     uint64
	DegU       int
	MaxLevel   int
	Entrypoint uint64
	Tombstones []uint64 // bitmap over ids
}

// SyncFromCPU uploads a snapshot (PostStartup, and after compaction /
// tombstone cleanup, or to recover a stale mirror).  Rows added after the
// snapshot must be re-applied with Add's propagation by the caller holding
// the CPU index's insert lock.
func (g *Index) SyncFromCPU(s *Snapshot) error {
	g.mu.Lock()
	defer g.mu.Unlock()
	g.stale.Store(true)
	if s.N > g.capacity {
		return errors.Errorf("wvgpu: snapshot of %d nodes exceeds capacity %d", s.N, g.capacity)
	}
	if s.N > 0 {
		if rc := C.wv_index_upload_vectors(g.ix, (*C.float)(unsafe.Pointer(&s.Vectors[0])), C.uint64_t(s.N), 0); rc != 0 {
			return lastErr("upload vectors", rc)
		}
		var upper *C.uint32_t
		if len(s.Upper) > 0 {
			upper = (*C.uint32_t)(unsafe.Pointer(&s.Upper[0]))
		}
		if rc := C.wv_index_upload_graph(g.ix, C.uint64_t(s.N), (*C.int8_t)(unsafe.Pointer(&s.Levels[0])),
			(*C.uint32_t)(unsafe.Pointer(&s.Layer0[0])), C.int(s.Deg0), (*C.uint32_t)(unsafe.Pointer(&s.UpperRow[0])),
			upper, C.uint64_t(s.NUpper), C.int(s.DegU), C.int(s.MaxLevel), C.uint64_t(s.Entrypoint)); rc != 0 {
			return lastErr("upload graph", rc)
		}
	}
	var tb *C.uint64_t
	if len(s.Tombstones) > 0 {
		tb = (*C.uint64_t)(unsafe.Pointer(&s.Tombstones[0]))
	}
	if rc := C.wv_index_set_tombstones(g.ix, tb, C.uint64_t(len(s.Tombstones)*64)); rc != 0 {
		return lastErr("tombstones", rc)
	}
	g.stale.Store(false)
	return nil
}

func (g *Index) close() {
	g.mu.Lock()
	defer g.mu.Unlock()
	if g.b != nil {
		C.wv_batcher_destroy(g.b) // drains waiting searches first
		g.b = nil
	}
	if g.ix != nil {
		C.wv_index_destroy(g.ix)
		g.ix = nil
	}
	g.stale.Store(true)
}

func (g *Index) Shutdown(ctx context.Context) error {
	g.close()
	return g.cpuIndex.Shutdown(ctx)
}

func (g *Index) Drop(ctx context.Context) error {
	g.close()
	return g.cpuIndex.Drop(ctx)
}
