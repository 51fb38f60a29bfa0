"""Shape descriptors for Keras-style shape inference (reference: S/utils/Shape.scala)."""


class Shape:
    @staticmethod
    def of(*dims):
        if len(dims) == 1 and isinstance(dims[0], (list, tuple)):
            if dims[0] and isinstance(dims[0][0], Shape):
                return MultiShape(list(dims[0]))
            return SingleShape(list(dims[0]))
        if dims and isinstance(dims[0], Shape):
            return MultiShape(list(dims))
        return SingleShape(list(dims))


class SingleShape(Shape):
    def __init__(self, dims):
        self.dims = [None if d is None or d == -1 else int(d) for d in dims]

    def toSingle(self):
        return list(self.dims)

    def toMulti(self):
        return [self]

    def copyAndUpdate(self, dim, v):
        d = list(self.dims)
        d[dim] = v
        return SingleShape(d)

    def __eq__(self, o):
        return isinstance(o, SingleShape) and o.dims == self.dims

    def __repr__(self):
        return f"SingleShape({self.dims})"


class MultiShape(Shape):
    def __init__(self, shapes):
        self.shapes = list(shapes)

    def toSingle(self):
        raise ValueError("MultiShape cannot be converted to a single shape")

    def toMulti(self):
        return list(self.shapes)

    def __eq__(self, o):
        return isinstance(o, MultiShape) and o.shapes == self.shapes

    def __repr__(self):
        return f"MultiShape({self.shapes})"
