from .folder import DatasetFromFolder, DevicePairCache, get_test_set, get_training_set
from .generate import compress, crop, generate_patches
from .image_io import is_image_file, load_img, normalize, save_img, tensor2img, tensor2np, to_tensor
from .synthetic import SyntheticPairs

__all__ = [n for n in dir() if not n.startswith("_")]
