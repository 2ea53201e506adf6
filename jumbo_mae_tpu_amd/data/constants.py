"""ImageNet normalization constants (reference /root/reference/src/dataset.py:37-38).

Normalization is applied on the device after the uint8 upload (pretraining.py:90-91)."""

IMAGENET_DEFAULT_MEAN = (0.485, 0.456, 0.406)
IMAGENET_DEFAULT_STD = (0.229, 0.224, 0.225)
