"""CPU oracle for the isotope trace simulator — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU and independently of the product code under
``istio-isotope_amd/``, the reference algorithm of the hot path:

* ``gounits``   — the Go/third-party arithmetic the graph loader relies on
                  (go-units v0.4.0 ``RAMInBytes``/``BytesSize``, Go
                  ``time.ParseDuration``/``Duration.String``,
                  ``strconv.ParseFloat`` syntax, ``pct.Percentage``).
* ``graph_ref`` — ``(*graph.ServiceGraph).UnmarshalJSON`` with the
                  ``defaults`` mechanism and ``validate``
                  (isotope/convert/pkg/graph/unmarshal.go:30-112,
                  validation.go:28-82, svc/unmarshal.go:29-41,
                  script/*.go, size/byte_size.go, pct/percentage.go,
                  svctype/service_type.go).
* ``philox``    — Philox4x32-10 (Random123 constants), pinned by the
                  Random123 known-answer vectors.
* ``executor_py`` — pure-Python recursive restatement of the script executor
                  (isotope/service/pkg/srv/handler.go:37-79,
                  executable.go:43-179) in virtual integer-ns time, for small
                  cases.
* ``isim_oracle.c`` (+ ``executor.py`` ctypes wrapper) — the same executor in
                  plain C with OpenMP, used for larger parity cases and as the
                  ``cpu_baseline`` leg of ``bench.py``.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker. The
product path never routes through it.

Parity status: the loader restatement is pinned by the reference's own Go
test vectors (transcribed into ``tests/golden/``). The executor semantics are
NOT pinned by any reference test (``service/pkg/srv`` has zero tests and the
reference is Go, which cannot be built here); they are pinned by the
hand-derived known-answer tests of SURVEY.md Appendix B and by the
pure-Python / C cross-check. See DESIGN.md §"Oracle and parity".
"""
