"""AIR configs of the reference's ``air`` crate, encoded for the GPU quotient.

Mirrors ``AirPermutationConfig`` (air/src/air_permutation.rs:1-24),
``AirLookupConfig`` (air/src/air_lookup.rs:1-40), ``AirConfig`` and
``LineaAIR`` (air/src/lib.rs:11-54).  ``LineaAIR.descriptor()`` produces the
int32 descriptor of include/lsp.h that the quotient kernel interprets with
the constraint order of ``LineaAIR::eval`` (air/src/lib.rs:47-167).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Union

LSP_AIR_PERMUTATION, LSP_AIR_LOOKUP = 1, 2


@dataclass
class AirPermutationConfig:
    a_columns_ids: List[int]
    b_columns_ids: List[int]
    b_inverse_id: int
    check_id: int

    def shift(self, shift: int) -> None:
        self.a_columns_ids = [i + shift for i in self.a_columns_ids]
        self.b_columns_ids = [i + shift for i in self.b_columns_ids]
        self.b_inverse_id += shift
        self.check_id += shift

    def width(self) -> int:
        return len(self.a_columns_ids) + len(self.b_columns_ids) + 2

    def encode(self) -> List[int]:
        return ([LSP_AIR_PERMUTATION, len(self.a_columns_ids), len(self.b_columns_ids)]
                + list(self.a_columns_ids) + list(self.b_columns_ids) + [self.b_inverse_id, self.check_id])


@dataclass
class AirLookupConfig:
    a_columns_ids: List[int]
    b_columns_ids: List[List[int]]
    a_filter_id: int
    b_filter_id: List[int]
    a_inverses_id: int
    b_inverses_id: List[int]
    occurrences_id: List[int]
    check_id: int

    def shift(self, shift: int) -> None:
        self.a_columns_ids = [i + shift for i in self.a_columns_ids]
        self.b_columns_ids = [[i + shift for i in t] for t in self.b_columns_ids]
        self.a_filter_id += shift
        self.b_filter_id = [i + shift for i in self.b_filter_id]
        self.a_inverses_id += shift
        self.b_inverses_id = [i + shift for i in self.b_inverses_id]
        self.occurrences_id = [i + shift for i in self.occurrences_id]
        self.check_id += shift

    def width(self) -> int:
        return len(self.a_columns_ids) + len(self.b_columns_ids) * (len(self.b_columns_ids[0]) + 3) + 3

    def encode(self) -> List[int]:
        nt, nbc = len(self.b_columns_ids), len(self.b_columns_ids[0])
        out = [LSP_AIR_LOOKUP, len(self.a_columns_ids)] + list(self.a_columns_ids) + [nt, nbc]
        for t in self.b_columns_ids:
            assert len(t) == nbc, "all B tables must have the same number of columns"
            out += list(t)
        return (out + [self.a_filter_id] + list(self.b_filter_id) + [self.a_inverses_id]
                + list(self.b_inverses_id) + list(self.occurrences_id) + [self.check_id])


AirConfig = Union[AirLookupConfig, AirPermutationConfig]


@dataclass
class LineaAIR:
    configs: List[AirConfig] = field(default_factory=list)

    @property
    def width(self) -> int:
        return sum(c.width() for c in self.configs)

    def descriptor(self) -> List[int]:
        out = [len(self.configs)]
        for c in self.configs:
            out += c.encode()
        return out

    @staticmethod
    def from_descriptor(d: List[int]) -> "LineaAIR":
        it = iter(d)
        n = next(it)
        cfgs: List[AirConfig] = []
        for _ in range(n):
            t = next(it)
            if t == LSP_AIR_PERMUTATION:
                na, nb = next(it), next(it)
                a = [next(it) for _ in range(na)]
                b = [next(it) for _ in range(nb)]
                cfgs.append(AirPermutationConfig(a, b, next(it), next(it)))
            elif t == LSP_AIR_LOOKUP:
                na = next(it)
                a = [next(it) for _ in range(na)]
                nt, nbc = next(it), next(it)
                b = [[next(it) for _ in range(nbc)] for _ in range(nt)]
                af = next(it)
                bf = [next(it) for _ in range(nt)]
                ai = next(it)
                bi = [next(it) for _ in range(nt)]
                oc = [next(it) for _ in range(nt)]
                cfgs.append(AirLookupConfig(a, b, af, bf, ai, bi, oc, next(it)))
            else:
                raise ValueError(f"unknown AIR config type {t}")
        assert next(it, None) is None, "trailing data in AIR descriptor"
        return LineaAIR(cfgs)


def permutation_air(ncols: int) -> LineaAIR:
    """The benchmark AIR: one permutation group of ncols 'from' + ncols 'to'
    columns (trace/src/permutation.rs:81-90 column layout)."""
    return LineaAIR([AirPermutationConfig(list(range(ncols)), list(range(ncols, 2 * ncols)), 2 * ncols,
                                          2 * ncols + 1)])
