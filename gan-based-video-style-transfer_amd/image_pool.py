"""ImagePool — mirror of methods/GAN-based/CycleGANCon/util/image_pool.py:5-54.

History buffer of generated images for the discriminator update.  Same policy (fill to pool_size,
then with p=0.5 return a stored image and replace it with the new one), same use of Python's
global ``random`` (so runs are reproducible with random.seed).  Works on any leading-batch tensor
layout (the HIP model passes NHWC4 images); stored images stay resident on the GPU.
"""
import random

import torch


class ImagePool:
    def __init__(self, pool_size):
        self.pool_size = pool_size
        if self.pool_size > 0:
            self.num_imgs = 0
            self.images = []

    def query(self, images):
        if self.pool_size == 0:
            return images
        return_images = []
        for image in images:
            image = torch.unsqueeze(image.data, 0)
            if self.num_imgs < self.pool_size:
                self.num_imgs = self.num_imgs + 1
                self.images.append(image)
                return_images.append(image)
            else:
                p = random.uniform(0, 1)
                if p > 0.5:
                    random_id = random.randint(0, self.pool_size - 1)
                    tmp = self.images[random_id].clone()
                    self.images[random_id] = image
                    return_images.append(tmp)
                else:
                    return_images.append(image)
        return torch.cat(return_images, 0)
