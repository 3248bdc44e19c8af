"""Neural-type descriptors used by the encoder's input_types / output_types (reference
nemo/core/neural_types).  Descriptive only: axes + element type name."""
from __future__ import annotations


class ElementType:
    def __repr__(self):
        return type(self).__name__


class SpectrogramType(ElementType):
    pass


class LengthsType(ElementType):
    pass


class AcousticEncodedRepresentation(ElementType):
    pass


class LogprobsType(ElementType):
    pass


class LabelsType(ElementType):
    pass


class LossType(ElementType):
    pass


class NeuralType:
    def __init__(self, axes=None, elements_type=None, optional: bool = False):
        self.axes = tuple(axes) if axes is not None else None
        self.elements_type = elements_type
        self.optional = optional

    def __repr__(self):
        return f"NeuralType(axes={self.axes}, elements_type={self.elements_type!r}, optional={self.optional})"


class AudioSignal(ElementType):
    def __init__(self, freq=None):
        self.freq = freq


class MelSpectrogramType(SpectrogramType):
    pass


class EmbeddedTextType(ElementType):
    pass


class HypothesisType(ElementType):
    pass
