// Package isim runs isotope service-graph scripts for many request traces on
// an MI355X through libisim (include/isim.h): the cgo binding a maintainer
// adds next to isotope/service/pkg/srv (graph.go:34 HandlerFromServiceGraphYAML,
// handler.go:37 ServeHTTP) and isotope/convert/pkg (graph decoding, graphviz,
// kubernetes).  Build: make -C istio-isotope_amd/csrc (libisim.so), then
// `go build ./...` in go/ (needs a Go toolchain and sigs.k8s.io/yaml v1.2.0,
// the reference's own pin, isotope/go.mod:17).
package isim

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../istio-isotope_amd/isim -lisim -Wl,-rpath,${SRCDIR}/../../istio-isotope_amd/isim
#include <stdlib.h>
#include "isim.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"unsafe"

	"sigs.k8s.io/yaml"
)

type Graph struct{ g *C.isim_graph }
type Handler struct{ h *C.isim_handler }
type Params = C.isim_params
type TraceRecord = C.isim_trace_rec

func lastErr(rc C.int) error {
	if rc == C.ISIM_OK {
		return nil
	}
	return fmt.Errorf("isim status %d: %s", int(rc), C.GoString(C.isim_last_error()))
}

// GraphFromYAML mirrors yaml.Unmarshal(bytes, &graph.ServiceGraph{}):
// sigs.k8s.io/yaml converts to JSON, libisim applies UnmarshalJSON.
func GraphFromYAML(b []byte) (*Graph, error) {
	j, err := yaml.YAMLToJSON(b)
	if err != nil {
		return nil, err
	}
	if len(j) == 0 {
		return nil, errors.New("empty graph")
	}
	var g *C.isim_graph
	rc := C.isim_graph_unmarshal_json((*C.char)(unsafe.Pointer(&j[0])), C.size_t(len(j)), &g)
	if rc != C.ISIM_OK {
		return nil, lastErr(rc)
	}
	return &Graph{g}, nil
}

func (g *Graph) Close() { C.isim_graph_free(g.g) }

// NewHandler mirrors srv.HandlerFromServiceGraphYAML(path, serviceName);
// serviceName "" selects the first isEntrypoint service.
func NewHandler(g *Graph, serviceName string, p Params) (*Handler, error) {
	var name *C.char
	if serviceName != "" {
		name = C.CString(serviceName)
		defer C.free(unsafe.Pointer(name))
	}
	var h *C.isim_handler
	if rc := C.isim_handler_create(g.g, name, &p, &h); rc != C.ISIM_OK {
		return nil, lastErr(rc)
	}
	return &Handler{h}, nil
}

// Serve simulates traces [begin, begin+len(recs)) on GPU `device`; stats is
// resized to the handler's stats words.
func (h *Handler) Serve(device int, begin uint64, recs []TraceRecord) ([]uint64, error) {
	var info C.isim_handler_info
	if rc := C.isim_handler_info_get(h.h, &info); rc != C.ISIM_OK {
		return nil, lastErr(rc)
	}
	stats := make([]uint64, int(info.stats_words))
	var rp *TraceRecord
	if len(recs) > 0 {
		rp = &recs[0]
	}
	rc := C.isim_serve(h.h, C.int(device), C.uint64_t(begin), C.uint64_t(len(recs)), rp,
		u64ptr(stats))
	return stats, lastErr(rc)
}

func (h *Handler) Close() { C.isim_handler_free(h.h) }

// MarshalJSON returns json.Marshal(graph) as Go would produce it; DOT the
// `isotope convert graphviz` text.
func (g *Graph) text(f func(*C.isim_graph, *C.char, C.size_t, *C.size_t) C.int) (string, error) {
	var n C.size_t
	if rc := f(g.g, nil, 0, &n); rc != C.ISIM_OK {
		return "", lastErr(rc)
	}
	buf := make([]byte, int(n))
	if rc := f(g.g, (*C.char)(unsafe.Pointer(&buf[0])), n, &n); rc != C.ISIM_OK {
		return "", lastErr(rc)
	}
	return string(buf[:len(buf)-1]), nil
}
func (g *Graph) MarshalJSON() ([]byte, error) {
	s, err := g.text(func(a *C.isim_graph, b *C.char, c C.size_t, d *C.size_t) C.int {
		return C.isim_graph_marshal_json(a, b, c, d)
	})
	return []byte(s), err
}
func (g *Graph) DOT() (string, error) {
	return g.text(func(a *C.isim_graph, b *C.char, c C.size_t, d *C.size_t) C.int {
		return C.isim_graph_to_dot(a, b, c, d)
	})
}

// ServeUnderLoad runs the per-replica worker-pool DES (config 5) for
// len(recs) open-loop arrivals with the given mean gap.
func (h *Handler) ServeUnderLoad(device int, begin uint64, meanGapNs uint64, recs []TraceRecord) (stats, table []uint64, err error) {
	var info C.isim_handler_info
	var dinfo C.isim_des_info
	if rc := C.isim_handler_info_get(h.h, &info); rc != C.ISIM_OK {
		return nil, nil, lastErr(rc)
	}
	if rc := C.isim_des_info_get(h.h, &dinfo); rc != C.ISIM_OK {
		return nil, nil, lastErr(rc) // outside the DES graph class: the reason is in the message
	}
	stats = make([]uint64, int(info.stats_words))
	table = make([]uint64, int(dinfo.table_rows)*C.ISIM_DES_ROW_WORDS+1)
	p := C.isim_des_params{mean_interarrival_ns: C.uint64_t(meanGapNs)}
	var rp *TraceRecord
	if len(recs) > 0 {
		rp = &recs[0]
	}
	// 32-bit rows; a batch with a latency >= 2^31 ns is rerun with 64-bit rows inside the call
	rc := C.isim_serve_des(h.h, C.int(device), &p, C.uint64_t(begin), C.uint64_t(len(recs)), rp,
		u64ptr(stats), u64ptr(table))
	return stats, table, lastErr(rc)
}

// DesBatch is the item engine's report on the handler's last DES batch
// (isim_des_last_batch): passes over the rounds, host synchronisations,
// executed invocations.
type DesBatch struct {
	Passes, Syncs uint32
	Items         uint64
}

// LastDesBatch reports the item engine's last batch (zero before the first).
func (h *Handler) LastDesBatch() (DesBatch, error) {
	var st C.isim_des_batch_stats
	if rc := C.isim_des_last_batch(h.h, &st); rc != C.ISIM_OK {
		return DesBatch{}, lastErr(rc)
	}
	return DesBatch{uint32(st.passes), uint32(st.syncs), uint64(st.items)}, nil
}

type Multi struct{ m *C.isim_multi }

// u64ptr passes an empty slice as NULL (libisim then reports EINVAL) instead
// of panicking on &s[0].
func u64ptr(s []uint64) *C.uint64_t {
	if len(s) == 0 {
		return nil
	}
	return (*C.uint64_t)(unsafe.Pointer(&s[0]))
}

// NewMultiNode drives every listed device from this process (ncclCommInitAll).
func NewMultiNode(devices []int32) (*Multi, error) {
	var m *C.isim_multi
	if len(devices) == 0 {
		return nil, lastErr(C.isim_multi_init_all(nil, 0, &m)) // libisim's EINVAL and message
	}
	rc := C.isim_multi_init_all((*C.int)(unsafe.Pointer(&devices[0])), C.int(len(devices)), &m)
	return &Multi{m}, lastErr(rc)
}

// MultiPrecheck makes the local checks of NewMultiRank (RCCL loads, the
// device can be selected) before the collective creation, so the ranks can
// agree on them out of band first.
func MultiPrecheck(device int) error { return lastErr(C.isim_multi_precheck(C.int(device))) }

// MultiID is created on rank 0 and shipped to the other ranks (e.g. over gRPC).
func MultiID() ([128]byte, error) {
	var id C.isim_multi_id
	rc := C.isim_multi_get_id(&id)
	return *(*[128]byte)(unsafe.Pointer(&id)), lastErr(rc)
}

func NewMultiRank(id [128]byte, nRanks, rank, device int) (*Multi, error) {
	var m *C.isim_multi
	rc := C.isim_multi_init_rank((*C.isim_multi_id)(unsafe.Pointer(&id)), C.int(nRanks), C.int(rank),
		C.int(device), &m)
	return &Multi{m}, lastErr(rc)
}

func (m *Multi) Close() { C.isim_multi_free(m.m) }

// ServeSharded walks this process's shards of [begin, begin + nRanks*perRank)
// and returns the node-wide merged stats (identical on every rank).
func (h *Handler) ServeSharded(m *Multi, begin, perRank uint64, recs []TraceRecord) ([]uint64, error) {
	var info C.isim_handler_info
	if rc := C.isim_handler_info_get(h.h, &info); rc != C.ISIM_OK {
		return nil, lastErr(rc)
	}
	stats := make([]uint64, int(info.stats_words))
	var rp *TraceRecord
	if len(recs) > 0 {
		rp = &recs[0] // n_local * perRank records
	}
	rc := C.isim_serve_multi(h.h, m.m, C.uint64_t(begin), C.uint64_t(perRank), rp,
		u64ptr(stats))
	return stats, lastErr(rc)
}

// Abort makes the peers' pending or next collectives fail (isim_multi_abort)
// instead of waiting for a rank that failed before a collective.
func (m *Multi) Abort() error { return lastErr(C.isim_multi_abort(m.m)) }

// K8sOptions are the arguments of kubernetes.ServiceGraphToKubernetesManifests
// (isotope/convert/pkg/kubernetes/kubernetes.go:56-63) plus the two EXT
// determinism knobs (creationTimestamp, RBAC rule names).
type K8sOptions struct {
	ServiceNodeSelector              map[string]string
	ServiceImage                     string
	ServiceMaxIdleConnectionsPerHost int
	ClientNodeSelector               map[string]string
	ClientImage                      string
	EnvironmentName                  string // "NONE" or "ISTIO"
	CreationTimestampUnix            int64
	RbacSeed                         uint64
}

func cStrings(m map[string]string) (**C.char, C.int32_t, func()) {
	if len(m) == 0 {
		return nil, 0, func() {}
	}
	arr := C.malloc(C.size_t(2*len(m)) * C.size_t(unsafe.Sizeof(uintptr(0))))
	ptrs := (*[1 << 28]*C.char)(arr)[: 2*len(m) : 2*len(m)]
	i := 0
	for k, v := range m {
		ptrs[i], ptrs[i+1] = C.CString(k), C.CString(v)
		i += 2
	}
	return (**C.char)(arr), C.int32_t(len(m)), func() {
		for _, p := range ptrs {
			C.free(unsafe.Pointer(p))
		}
		C.free(arr)
	}
}

// KubernetesManifests mirrors kubernetes.ServiceGraphToKubernetesManifests.
func (g *Graph) KubernetesManifests(o K8sOptions) ([]byte, error) {
	var p C.isim_k8s_params
	si, ci, env := C.CString(o.ServiceImage), C.CString(o.ClientImage), C.CString(o.EnvironmentName)
	defer C.free(unsafe.Pointer(si))
	defer C.free(unsafe.Pointer(ci))
	defer C.free(unsafe.Pointer(env))
	ss, sn, sfree := cStrings(o.ServiceNodeSelector)
	defer sfree()
	cs, cn, cfree := cStrings(o.ClientNodeSelector)
	defer cfree()
	p.service_image, p.client_image, p.environment_name = si, ci, env
	p.service_node_selector, p.n_service_node_selector = ss, sn
	p.client_node_selector, p.n_client_node_selector = cs, cn
	p.service_max_idle_connections_per_host = C.int32_t(o.ServiceMaxIdleConnectionsPerHost)
	p.creation_timestamp_s = C.int64_t(o.CreationTimestampUnix)
	p.rbac_seed = C.uint64_t(o.RbacSeed)
	s, err := g.text(func(a *C.isim_graph, b *C.char, c C.size_t, d *C.size_t) C.int {
		return C.isim_graph_to_k8s_manifests(a, &p, b, c, d)
	})
	return []byte(s), err
}

// MarshalYAML returns yaml.Marshal(graph) as sigs.k8s.io/yaml renders it.
func (g *Graph) MarshalYAML() ([]byte, error) {
	s, err := g.text(func(a *C.isim_graph, b *C.char, c C.size_t, d *C.size_t) C.int {
		return C.isim_graph_marshal_yaml(a, b, c, d)
	})
	return []byte(s), err
}
