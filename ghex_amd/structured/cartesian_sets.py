"""ghex_amd.structured.cartesian_sets — the index-set vocabulary of the reference Python binding
(bindings/python/src/ghex/structured/cartesian_sets.py), so code and tests written against
`ghex.structured.cartesian_sets` run unchanged: `UnitRange` (integers start <= i < stop, either
end may be +-inf), `ProductSet` (a box: the product of UnitRanges), their unions (`union`,
`UnionRange`, `UnionCartesian`) and `IndexSpace` (labelled subsets of one grid, `decompose`).

Setup-time host helpers only (domain boxes, halo regions, decompositions; the device path never
sees them). Unlike the reference, a union is always kept as disjoint primitives: every element is
held once, so `size`, iteration and the set operations are exact for any overlap (`disjoint=`
is accepted for compatibility and has nothing left to promise). `simplify=True` merges pieces
that share a face into one box where they form one; equality is set equality either way."""
from __future__ import annotations

import itertools
import math
import warnings
from typing import Any, Callable, Dict, Sequence, Tuple

INF = math.inf


def is_integer_like(v) -> bool:
    return isinstance(v, int) or v in (INF, -INF)


class Set:
    """Base of every index set: equality is set equality."""

    def __eq__(self, other):
        if not isinstance(other, Set):
            return False
        return self.issubset(other) and other.issubset(self)

    def __ne__(self, other):
        return not self == other

    def issubset(self, other: "Set") -> bool:
        return self.without(other).empty


# ---- integers -------------------------------------------------------------------------------

class IntegerSet(Set):
    @staticmethod
    def empty_set() -> "UnitRange":
        return UnitRange(0, 0)

    @staticmethod
    def universe() -> "UnitRange":
        return UnitRange(-INF, INF)

    @staticmethod
    def primitive_type():
        return UnitRange

    @staticmethod
    def union_type():
        return UnionRange

    def simplify(self) -> "IntegerSet":
        return self


class UnitRange(IntegerSet):
    """The integers start <= i < stop. An empty range is stored as (0, 0)."""

    def __init__(self, start, stop):
        if not (is_integer_like(start) and is_integer_like(stop)):
            raise TypeError(f"UnitRange bounds must be integers or +-inf, got {start!r}, {stop!r}")
        if stop < start:
            raise ValueError(f"UnitRange: stop {stop} < start {start}")
        self.start, self.stop = (0, 0) if start == stop else (start, stop)

    # -- size and shape
    @property
    def size(self):
        return self.stop - self.start

    def __len__(self):
        if math.isinf(self.size):
            raise OverflowError("unbounded UnitRange has no length")
        return int(self.size)

    @property
    def empty(self) -> bool:
        return self.start >= self.stop

    @property
    def bounds(self) -> "UnitRange":
        return self

    def elements(self):
        return [] if self.empty else [self]

    # -- element access
    def __contains__(self, i) -> bool:
        return self.start <= i < self.stop

    def __iter__(self):
        if math.isinf(self.start) or math.isinf(self.stop):
            raise ValueError("cannot iterate an unbounded UnitRange")
        return iter(range(self.start, self.stop))

    def __getitem__(self, arg):
        if isinstance(arg, slice):
            if arg.step not in (None, 1):
                raise ValueError("UnitRange slices have step 1")

            def at(k, default):
                if k is None:
                    return default
                return (self.stop if k < 0 else self.start) + k
            return UnitRange(at(arg.start, self.start), at(arg.stop, self.stop))
        if isinstance(arg, int):
            v = (self.stop if arg < 0 else self.start) + arg
            if v not in self:
                raise IndexError(arg)
            return v
        raise ValueError(f"invalid UnitRange index {arg!r}")

    # -- set algebra
    def intersect(self, other: Set) -> IntegerSet:
        if isinstance(other, UnitRange):
            lo = max(self.start, other.start)
            return UnitRange(lo, max(lo, min(self.stop, other.stop)))
        if isinstance(other, UnionRange):
            return other.intersect(self)
        raise TypeError(f"cannot intersect a UnitRange with {type(other).__name__}")

    def _minus(self, other: "UnitRange") -> list:
        """self \\ other as at most two UnitRanges."""
        if self.intersect(other).empty:
            return self.elements()
        return [r for r in (UnitRange(self.start, max(self.start, other.start)),
                            UnitRange(min(self.stop, other.stop), self.stop)) if not r.empty]

    def without(self, *others: Set, simplify: bool = True) -> IntegerSet:
        pieces = self.elements()
        for o in others:
            for e in o.elements():
                pieces = [p for q in pieces for p in q._minus(e)]
        return union(*pieces, simplify=simplify) if pieces else UnitRange(0, 0)

    def complement(self, other: Set = None, simplify: bool = True) -> IntegerSet:
        return (other if other is not None else self.universe()).without(self, simplify=simplify)

    def union(self, *others: Set) -> IntegerSet:
        return union(self, *others)

    def extend(self, arg) -> "UnitRange":
        if self.empty:
            return self
        lo, hi = (arg, arg) if isinstance(arg, int) else arg
        return UnitRange(self.start - lo, self.stop + hi)

    def translate(self, arg: int) -> "UnitRange":
        return self if self.empty else UnitRange(self.start + arg, self.stop + arg)

    def as_tuple(self) -> Tuple:
        return self.start, self.stop

    def __mul__(self, other):
        """Cartesian product: UnitRange * UnitRange / ProductSet / a union of either."""
        if isinstance(other, UnitRange):
            return ProductSet(self, other)
        if isinstance(other, ProductSet):
            return ProductSet(self, *other.args)
        if isinstance(other, (UnionRange, UnionCartesian)):
            return union(*(self * a for a in other.args), simplify=False)
        return NotImplemented

    def __hash__(self):
        return hash((self.start, self.stop))

    def __repr__(self):
        return f"UnitRange({self.start}, {self.stop})"

    __str__ = __repr__


# ---- boxes ----------------------------------------------------------------------------------

class CartesianSet(Set):
    """A set of integer tuples of one dimensionality."""

    @property
    def dim(self) -> int:
        warnings.warn("`dim` is deprecated, use `ndim` instead.", DeprecationWarning, stacklevel=2)
        return self.ndim

    def empty_set(self) -> "ProductSet":
        return ProductSet(*([UnitRange(0, 0)] * self.ndim))

    def universe(self) -> "ProductSet":
        return ProductSet(*([UnitRange(-INF, INF)] * self.ndim))

    @staticmethod
    def primitive_type():
        return ProductSet

    @staticmethod
    def union_type():
        return UnionCartesian

    @classmethod
    def from_range(cls, rng: IntegerSet) -> "CartesianSet":
        pieces = [ProductSet(r) for r in rng.elements()]
        return union(*pieces, simplify=False) if pieces else ProductSet(UnitRange(0, 0))

    def simplify(self) -> "CartesianSet":
        return self


class ProductSet(CartesianSet):
    """The box args[0] x args[1] x ... (UnitRanges), iterated with the LAST dimension fastest."""

    def __init__(self, *args: UnitRange):
        if not args or not all(isinstance(a, UnitRange) for a in args):
            raise TypeError("ProductSet takes one or more UnitRanges")
        self.args = tuple(args)

    @classmethod
    def from_coords(cls, first: Sequence[int], last: Sequence[int]) -> "ProductSet":
        """The box with inclusive corners first .. last."""
        return cls(*(UnitRange(int(f), int(l) + 1) for f, l in zip(first, last)))

    @property
    def ranges(self):
        return self.args

    @property
    def ndim(self) -> int:
        return len(self.args)

    @property
    def shape(self):
        return tuple(a.size for a in self.args)

    @property
    def size(self):
        return math.prod(self.shape)

    @property
    def empty(self) -> bool:
        return any(a.empty for a in self.args)

    @property
    def bounds(self) -> "ProductSet":
        return self

    def elements(self):
        return [] if self.empty else [self]

    def __contains__(self, idx) -> bool:
        if len(idx) != self.ndim:
            raise ValueError(f"{len(idx)}-tuple tested against a {self.ndim}-D set")
        return all(i in a for a, i in zip(self.args, idx))

    def __iter__(self):
        return itertools.product(*self.args)

    def __getitem__(self, idx):
        if isinstance(idx, (int, slice)):
            idx = (idx,)
        if len(idx) != self.ndim:
            raise IndexError(idx)
        if all(isinstance(i, int) for i in idx):
            return tuple(a[i] for a, i in zip(self.args, idx))
        if all(isinstance(i, slice) for i in idx):
            return ProductSet(*(a[i] for a, i in zip(self.args, idx)))
        raise ValueError(f"index with all integers or all slices, got {idx!r}")

    def intersect(self, other: CartesianSet) -> CartesianSet:
        if isinstance(other, ProductSet):
            self._same_dim(other)
            return ProductSet(*(a.intersect(b) for a, b in zip(self.args, other.args)))
        if isinstance(other, UnionCartesian):
            return other.intersect(self)
        raise TypeError(f"cannot intersect a ProductSet with {type(other).__name__}")

    def _minus(self, other: "ProductSet") -> list:
        """self \\ other as disjoint boxes: slabs peeled off dimension by dimension (at most two
        per dimension), the remainder narrowed to the overlap before the next dimension."""
        self._same_dim(other)
        if self.intersect(other).empty:
            return self.elements()
        out, cur = [], list(self.args)
        for d in range(self.ndim):
            for piece in cur[d]._minus(other.args[d]):
                out.append(ProductSet(*cur[:d], piece, *cur[d + 1:]))
            cur[d] = cur[d].intersect(other.args[d])
        return out

    def without(self, *others: CartesianSet, simplify: bool = True) -> CartesianSet:
        pieces = self.elements()
        for o in others:
            for e in o.elements():
                pieces = [p for q in pieces for p in q._minus(e)]
        return union(*pieces, simplify=simplify) if pieces else self.empty_set()

    def complement(self, other: CartesianSet = None, simplify: bool = True) -> CartesianSet:
        return (other if other is not None else self.universe()).without(self, simplify=simplify)

    def union(self, *others: CartesianSet) -> CartesianSet:
        return union(self, *others)

    def extend(self, *args) -> "ProductSet":
        if self.empty:
            return self
        if len(args) != self.ndim:
            raise ValueError("extend takes one halo (int or (minus, plus)) per dimension")
        return ProductSet(*(a.extend(h) for a, h in zip(self.args, args)))

    def translate(self, *args: int) -> "ProductSet":
        if len(args) != self.ndim:
            raise ValueError("translate takes one offset per dimension")
        return ProductSet(*(a.translate(t) for a, t in zip(self.args, args)))

    def as_tuple(self):
        return tuple(a.as_tuple() for a in self.args)

    def __mul__(self, other):
        if isinstance(other, UnitRange):
            return ProductSet(*self.args, other)
        if isinstance(other, ProductSet):
            return ProductSet(*self.args, *other.args)
        if isinstance(other, (UnionRange, UnionCartesian)):
            return union(*(self * a for a in other.args), simplify=False)
        return NotImplemented

    def _same_dim(self, other):
        if other.ndim != self.ndim:
            raise ValueError(f"{self.ndim}-D and {other.ndim}-D sets")

    def __hash__(self):
        return hash(self.args)

    def __repr__(self):
        return " * ".join(repr(a) for a in self.args)

    __str__ = __repr__


# ---- unions ---------------------------------------------------------------------------------

class _UnionOf:
    """A union of disjoint, non-empty primitives (UnitRanges or ProductSets), in order."""

    def __init__(self, *args, disjoint: bool = True):
        if len(args) < 2:
            raise ValueError("a union holds two or more pieces; use union() to build one")
        if not all(isinstance(a, self.primitive_type()) and not a.empty for a in args):
            raise ValueError("a union holds non-empty primitive sets; use union() to build one")
        self.args = tuple(args)
        self.disjoint = True

    @property
    def size(self):
        return sum(a.size for a in self.args)

    @property
    def empty(self) -> bool:
        return False

    def elements(self):
        return list(self.args)

    def __iter__(self):
        for a in self.args:
            yield from a

    def __contains__(self, x) -> bool:
        return any(x in a for a in self.args)

    def intersect(self, other: Set):
        pieces = [p for a in self.args for p in a.intersect(other).elements()]
        return union(*pieces, simplify=False) if pieces else self.empty_set()

    def without(self, *others: Set, simplify: bool = True):
        pieces = [p for a in self.args for p in a.without(*others, simplify=False).elements()]
        return union(*pieces, simplify=simplify) if pieces else self.empty_set()

    def complement(self, other: Set = None, simplify: bool = True):
        return (other if other is not None else self.universe()).without(self, simplify=simplify)

    def union(self, *others: Set):
        return union(self, *others)

    def translate(self, *args: int):
        return union(*(a.translate(*args) for a in self.args), simplify=False)

    def simplify(self):
        return _merge(list(self.args))

    def make_disjoint(self):
        return self

    def __hash__(self):
        return hash(frozenset(self.args))

    def __repr__(self):
        return "union(" + ", ".join(repr(a) for a in self.args) + ")"

    __str__ = __repr__


class UnionRange(_UnionOf, IntegerSet):
    """A union of disjoint UnitRanges."""

    @property
    def bounds(self) -> UnitRange:
        return UnitRange(min(a.start for a in self.args), max(a.stop for a in self.args))

    def __mul__(self, other):
        return union(*(a * other for a in self.args), simplify=False)


class UnionCartesian(_UnionOf, CartesianSet):
    """A union of disjoint boxes of one dimensionality."""

    @property
    def ndim(self) -> int:
        return self.args[0].ndim

    @property
    def bounds(self) -> ProductSet:
        return ProductSet(*(UnitRange(min(a.args[d].start for a in self.args),
                                      max(a.args[d].stop for a in self.args))
                            for d in range(self.ndim)))

    @property
    def shape(self):
        return self.bounds.shape


def _merge(pieces: list):
    """Fuse pieces that share a face and agree in every other dimension, until none do."""
    changed = True
    while changed and len(pieces) > 1:
        changed = False
        for i in range(len(pieces)):
            for j in range(i + 1, len(pieces)):
                m = _fuse(pieces[i], pieces[j])
                if m is not None:
                    pieces[i] = m
                    del pieces[j]
                    changed = True
                    break
            if changed:
                break
    if len(pieces) == 1:
        return pieces[0]
    return pieces[0].union_type()(*pieces)


def _fuse(a, b):
    ra = a.args if isinstance(a, ProductSet) else (a,)
    rb = b.args if isinstance(b, ProductSet) else (b,)
    diff = [d for d in range(len(ra)) if ra[d].as_tuple() != rb[d].as_tuple()]
    if len(diff) != 1:
        return None
    d = diff[0]
    x, y = ra[d], rb[d]
    if x.stop == y.start or y.stop == x.start:
        r = UnitRange(min(x.start, y.start), max(x.stop, y.stop))
        if isinstance(a, ProductSet):
            return ProductSet(*ra[:d], r, *ra[d + 1:])
        return r
    return None


def union(*args: Set, simplify: bool = True, disjoint: bool = False) -> Set:
    """The union of index sets of one kind (integers or d-tuples): overlaps are removed (each
    later piece minus the earlier ones); one piece comes back as itself, none as the empty set."""
    if not args:
        raise ValueError("union() needs at least one set")
    first = args[0]
    pieces = []
    for a in args:
        for e in a.elements():
            new = [e]
            for p in pieces:
                new = [q for n in new for q in n._minus(p)]
            pieces.extend(new)
    if not pieces:
        return first.empty_set()
    if len(pieces) == 1:
        return pieces[0]
    if simplify:
        return _merge(pieces)
    return pieces[0].union_type()(*pieces)


# ---- labelled index spaces --------------------------------------------------------------------

class IndexSpace:
    """Labelled subsets of one grid; "definition" (the owned cells) is required."""

    def __init__(self, subset: Dict[Any, CartesianSet]):
        if "definition" not in subset:
            raise ValueError('an IndexSpace needs a "definition" subset')
        self.subset = dict(subset)

    @classmethod
    def from_sizes(cls, *shape: int) -> "IndexSpace":
        return cls({"definition": ProductSet(*(UnitRange(0, int(n)) for n in shape))})

    def __getitem__(self, idx):
        return self.subset["definition"][idx]

    def transform(self, fn: Callable[[CartesianSet], CartesianSet]) -> "IndexSpace":
        return IndexSpace({k: fn(v) for k, v in self.subset.items()})

    def intersect(self, mask: ProductSet) -> "IndexSpace":
        m = mask if mask.ndim == self.ndim else ProductSet(*mask.args[:self.ndim])
        return self.transform(lambda s: s.intersect(m))

    @property
    def covering(self) -> CartesianSet:
        return union(*self.subset.values(), simplify=False)

    @property
    def ndim(self) -> int:
        return self.subset["definition"].ndim

    @property
    def dim(self) -> int:
        warnings.warn("`dim` is deprecated, use `ndim` instead.", DeprecationWarning, stacklevel=2)
        return self.ndim

    @property
    def bounds(self) -> ProductSet:
        return self.covering.bounds

    @property
    def shape(self):
        return self.bounds.shape

    @property
    def default_origin(self):
        return tuple(a.start for a in self.subset["definition"].bounds.args)

    @property
    def empty(self) -> bool:
        return all(s.empty for s in self.subset.values())

    def translate(self, *offsets: int) -> "IndexSpace":
        return self.transform(lambda s: s.translate(*offsets))

    def prune(self) -> "IndexSpace":
        """Drop the empty subsets ("definition" stays, empty if it is)."""
        kept = {k: v.simplify() for k, v in self.subset.items() if not v.empty}
        kept.setdefault("definition", ProductSet(*([UnitRange(0, 0)] * self.ndim)))
        return IndexSpace(kept)

    def decompose(self, parts_per_dim: Sequence[int]) -> Dict[Tuple[int, ...], "IndexSpace"]:
        """Split every dimension into parts of floor(length / parts) cells (the last part takes
        the remainder), as the reference does; returns {part coordinate: IndexSpace} with every
        subset sliced to that part (subsets must be boxes)."""
        shape = self.covering.bounds.shape
        cuts = []
        for d, n in enumerate(parts_per_dim):
            step = int(shape[d]) // int(n)
            cuts.append([i * step for i in range(n)] + [int(shape[d])])
        out = {}
        for coord in itertools.product(*(range(n) for n in parts_per_dim)):
            sl = tuple(slice(cuts[d][c], cuts[d][c + 1]) for d, c in enumerate(coord))
            subs = {}
            for k, v in self.subset.items():
                if not isinstance(v, ProductSet):
                    raise TypeError(f"decompose slices box subsets only; {k!r} is a union")
                subs[k] = v[sl]
            out[coord] = IndexSpace(subs)
        return out

    def __repr__(self):
        return "IndexSpace(" + ", ".join(f"{k!r}: {v!r}" for k, v in self.subset.items()) + ")"


__all__ = ["Set", "IntegerSet", "UnitRange", "UnionRange", "CartesianSet", "ProductSet",
           "UnionCartesian", "IndexSpace", "union", "is_integer_like"]
