"""Device-side loader mirroring the reference CellDataset (dataset.py:21-361).

    CellDataset(data_dir, split='train', transform=None, max_size=1024, device='cuda')
    collate_fn(batch) -> {'images': [B,3,H,W] (device), 'batch_items': [...]}   # dataset.py:355-361

Same file split (sorted *.jpg, 70/15/15, dataset.py:37-51), the same resize-to-/32
sizes (:141-157), LabelMe 'live'/'dead' polygons scaled and truncated to int32 as the
reference does (:173-188), the semantic mask with later instances overwriting earlier
ones (:197-201), per-instance uint8 masks flipped with the image (:184-193, 209-222), the
cell-specific preprocessing of every split (:58-131, :204), and the training augmentations
drawn from Python's `random` in the reference's order, so a seeded run takes the same
decisions (:204-300).  Per pixel everything runs in HIP: polygon rasterisation, flips, the
numpy pixel ops (brightness, contrast, noise, gamma LUT -- bit-exact with the reference's
numpy lines), ToTensor (datapath.hip); LAB/HSV conversions, CLAHE, Sobel/Laplacian edge
features, GaussianBlur unsharp mask, filter2D sharpening (imgproc.hip).  Image decode stays
PIL on the host (I/O).

cv2 is absent from this image: cv2.fillPoly, cv2.resize and the cv2 colour / CLAHE / filter
calls are replaced by kernels that follow OpenCV's published algorithms (cv2.resize INTER_LINEAR
and RGB<->Lab 8U with OpenCV's own fixed-point arithmetic), pinned to the numpy restatements in
oracle/data_ref.py / oracle/imgproc_ref.py, not to cv2 (parity unpinned);
cv2.fillPoly is replaced by a documented fill rule.

Feeding the GPU (round 3): a sample makes no host round trip -- host arrays reach the device
through pinned staging buffers (ops.upload), the live ratio that selects the brightness /
contrast ranges is read on the device (eunet_augment_ratio_u8: the host draws the same
random.random() values random.uniform would).  The Gaussian noise is by default the reference's
own numpy draw (host_noise=True: np.random.normal, bit-exact values and np.random stream, one
synchronising copy per noisy sample); host_noise=False draws it on the device from a generator
seeded by one np.random draw -- sync-free and faster, same Python `random` decisions, but other
noise values and a shifted np.random stream.  DataLoader(workers=W, prefetch=P) decodes JPEG + JSON in W threads and runs the device
part of the next P batches on a side stream while the trainer consumes the current one; the
Python `random` draws stay in item order (one producer thread).
"""
from __future__ import annotations

import json
import multiprocessing
import os
import queue
import random
import threading
from collections import deque

import numpy as np
import torch

from . import ops


def reference_sizes(h: int, w: int, max_size: int):
    """dataset.py:141-157: target (h, w) multiples of 32."""
    if max(h, w) > max_size:
        scale = max_size / max(h, w)
        nh, nw = int(h * scale), int(w * scale)
        return (nh // 32) * 32, (nw // 32) * 32
    return (h // 32) * 32, (w // 32) * 32


def gamma_lut(gamma: float) -> np.ndarray:
    """dataset.py:273-275."""
    inv_gamma = 1.0 / gamma
    return np.array([((i / 255.0) ** inv_gamma) * 255 for i in np.arange(0, 256)]).astype(np.uint8)


def load_labelme(json_path: str, scale_h: float, scale_w: float):
    """dataset.py:161-195: (int32 polygons, labels 0 live / 1 dead, bboxes)."""
    with open(json_path, "r", encoding="utf-8") as f:
        ann = json.load(f)
    polys, labels, bboxes = [], [], []
    for shape in ann.get("shapes", []):
        label = shape["label"].lower()
        if label not in ("live", "dead"):
            continue
        pts = np.array(shape["points"], dtype=np.float32)
        pts[:, 0] *= scale_w
        pts[:, 1] *= scale_h
        pts = pts.astype(np.int32)
        polys.append(pts)
        labels.append(0 if label == "live" else 1)
        x_min, y_min = pts.min(axis=0)
        x_max, y_max = pts.max(axis=0)
        bboxes.append([x_min, y_min, x_max, y_max])
    return polys, labels, bboxes


def host_load(data_dir, name, max_size):
    """dataset.py:133-195 up to the pixels: JPEG decode (PIL), the /32 target size and the LabelMe
    polygons scaled to it.  Module level, so DataLoader worker processes can run it."""
    from PIL import Image
    image = np.array(Image.open(os.path.join(data_dir, name)).convert("RGB"))
    original_size = image.shape[:2]
    h, w = reference_sizes(*original_size, max_size)
    polys, labels, bboxes = load_labelme(os.path.join(data_dir, name.replace(".jpg", ".json")),
                                         h / original_size[0], w / original_size[1])
    return name, image, original_size, (h, w), polys, labels, bboxes


def _host_load_args(args):
    return host_load(*args)


class CellDataset:
    def __init__(self, data_dir: str, split: str = "train", transform=None, max_size: int = 1024,
                 device: str = "cuda", cell_preprocess: bool = True, host_noise: bool = True,
                 host_ratio: bool = False):
        self.data_dir, self.split, self.transform, self.max_size = data_dir, split, transform, max_size
        self.device = device
        self.cell_preprocess = cell_preprocess  # dataset.py:204 (always on in the reference)
        # host_noise (default): the reference's np.random.normal noise (exact values and np.random
        # stream; a host draw of 3 H W normals + one synchronising copy per noisy sample); False:
        # drawn on the device from a generator seeded by one np.random draw (sync-free; same Python
        # `random` decisions, other noise values)
        self.host_noise = host_noise
        # host_ratio: read the live ratio back to the host (round 2's path; one sync per sample)
        self.host_ratio = host_ratio
        self._noise_gen = None
        all_files = sorted(f for f in os.listdir(data_dir) if f.endswith(".jpg"))
        n_total = len(all_files)
        n_train, n_val = int(n_total * 0.7), int(n_total * 0.15)
        if split == "train":
            self.files = all_files[:n_train]
        elif split == "val":
            self.files = all_files[n_train:n_train + n_val]
        else:
            self.files = all_files[n_train + n_val:]

    def __len__(self):
        return len(self.files)

    @staticmethod
    def _apply_cell_specific_preprocessing(img, polys, labels):
        """dataset.py:58-131.  The live / dead unions of the instance masks (:93-100) are filled
        straight from the polygons (same fill rule as the instance masks)."""
        h, w, _ = img.shape
        live = [p for p, l in zip(polys, labels) if l == 0]
        dead = [p for p, l in zip(polys, labels) if l != 0]
        live_mask = ops.rasterize_polygons(live, [1] * len(live), h, w, img.device) if live else None
        dead_mask = ops.rasterize_polygons(dead, [1] * len(dead), h, w, img.device) if dead else None
        return ops.cell_preprocess_u8(img, live_mask, dead_mask)

    def _augment(self, img, mask):
        """dataset.py:204-294 in order; img HWC uint8 and mask int64 on the device.  Returns
        (img, mask, (flip_h, flip_v)): the flips are applied to the instance masks as well
        (dataset.py:212-213, 220-221), by rasterize_instances."""
        flip_h = flip_v = False
        if random.random() > 0.5:
            img, mask = ops.flip_u8(img, 1), ops.flip_mask(mask, 1)
            flip_h = True
        if random.random() > 0.5:
            img, mask = ops.flip_u8(img, 0), ops.flip_mask(mask, 0)
            flip_v = True
        counts = ops.semantic_counts(mask.reshape(1, -1), mask.reshape(1, -1))  # [1][class][0] = #pixels
        if self.host_ratio:
            c = counts[0, :, 0].tolist()
            total = c[1] + c[2]
            live_ratio = c[1] / total if total > 0 else 0.5
            if random.random() > 0.3:
                if live_ratio > 0.6:
                    alpha = random.uniform(0.8, 1.3)
                elif live_ratio < 0.4:
                    alpha = random.uniform(0.6, 1.1)
                else:
                    alpha = random.uniform(0.7, 1.3)
                ops.augment_u8(img, alpha=alpha)
            if random.random() > 0.3:
                beta = random.uniform(-20, 40) if live_ratio < 0.4 else random.uniform(-30, 30)
                ops.augment_u8(img, beta=beta)
        else:
            # every branch of the reference draws one uniform = a + (b - a) random.random(): draw
            # that random() here, let the device pick (a, b) from its own live ratio
            ua = random.random() if random.random() > 0.3 else None
            ub = random.random() if random.random() > 0.3 else None
            ops.augment_ratio_u8(img, counts, ua, ub)
        if random.random() > 0.5:  # HSV saturation (:259-264)
            ops.hsv_adjust_u8(img, sat=random.uniform(0.8, 1.3))
        if random.random() > 0.4:  # CLAHE on L (:267-272)
            img = ops.clahe_rgb_u8(img, random.uniform(1.5, 3.0))
        if random.random() > 0.5:
            sigma = random.uniform(3, 10)
            if self.host_noise:
                noise = np.random.normal(0, sigma, tuple(img.shape)).astype(np.float32)
                ops.augment_u8(img, noise=torch.from_numpy(noise).to(img.device))
            else:
                ops.augment_u8(img, noise=self._device_noise(sigma, tuple(img.shape), img.device))
        if random.random() > 0.5:
            lut = ops.upload(gamma_lut(random.uniform(0.7, 1.3)), img.device)
            ops.augment_u8(img, lut=lut)
        if random.random() > 0.6:  # sharpening (:287-292)
            img = ops.sharpen_u8(img, random.uniform(0.1, 0.3))
        if random.random() > 0.6:  # HSV jitter (:295-300): hue drawn before value
            hue = random.uniform(-10, 10)
            ops.hsv_adjust_u8(img, hue=hue, val=random.uniform(0.9, 1.1))
        return img, mask, (flip_h, flip_v)

    def _device_noise(self, sigma, shape, device):
        """N(0, sigma) float32 noise drawn on the device; the generator is reseeded from one
        np.random draw per use, so np.random.seed still makes a run reproducible."""
        if self._noise_gen is None:
            self._noise_gen = torch.Generator(device=device)
        self._noise_gen.manual_seed(int(np.random.randint(0, 2 ** 62, dtype=np.int64)))
        return torch.normal(0.0, float(sigma), shape, generator=self._noise_gen, device=device)

    def host_args(self, idx):
        """Picklable arguments of host_load for item idx (DataLoader worker processes)."""
        return self.data_dir, self.files[idx], self.max_size

    def load_host(self, idx):
        """The host half of __getitem__ (no GPU work, no random draws): the decoded image, the
        reference's target size and the scaled LabelMe polygons."""
        return host_load(*self.host_args(idx))

    def __getitem__(self, idx):
        return self.from_host(self.load_host(idx))

    def from_host(self, host):
        """The device half of __getitem__ (enqueued on the current stream, no host synchronisation
        unless host_noise / host_ratio)."""
        name, image, original_size, (h, w), polys, labels, bboxes = host
        img = ops.upload(image, self.device)
        if (h, w) != tuple(original_size):
            img = ops.resize_u8(img, h, w)
        mask = ops.rasterize_polygons(polys, [l + 1 for l in labels], h, w, img.device)
        if self.cell_preprocess:
            img = self._apply_cell_specific_preprocessing(img.contiguous(), polys, labels)
        flips = (False, False)
        if self.split == "train":
            img, mask, flips = self._augment(img.contiguous(), mask)
        instance_masks = list(ops.rasterize_instances(polys, h, w, img.device, flip_h=flips[0], flip_v=flips[1]))
        tensor = self.transform(img) if self.transform else ops.to_tensor(img)
        # dataset.py:313-321; bboxes stay in the unflipped frame, as the reference leaves them
        return {"image": tensor, "instance_masks": instance_masks, "instance_labels": labels, "bboxes": bboxes,
                "semantic_mask": mask, "image_id": name, "original_size": original_size}


def collate_fn(batch):
    """dataset.py:355-361."""
    return {"images": torch.stack([item["image"] for item in batch]), "batch_items": batch}


class DataLoader:
    """In-order / shuffled batch iterator over a CellDataset (the reference's train_model loaders,
    train_eval.py:1071-1075, run with num_workers=0).

    workers > 0: JPEG decode + JSON parsing (host_load) in that many worker processes (spawned:
    they never touch the GPU), in item order.  prefetch > 0: the device half of the next `prefetch`
    batches is enqueued on a side stream, from the calling thread, before the current batch is
    handed out; the caller's stream waits on each batch's event (no host synchronisation) and its
    tensors are recorded on that stream.  One thread issues every Python `random` draw in item
    order, so a seeded run takes the same augmentation decisions either way.  (A producer thread
    plus decode threads was tried first: its hundreds of short GIL-releasing launches per batch
    ping-ponged the GIL with the other threads -- slower than no prefetch, profiles/r03_loader.txt.)
    thread=True builds the device halves in one producer thread instead (DataLoader._threaded),
    for a consumer whose per-batch host work is one graph launch (Trainer.step_graph).
    Datasets without host_args / from_host run in the loop."""

    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False, collate_fn=collate_fn,
                 workers: int = 0, prefetch: int = 0, thread: bool = False):
        self.dataset, self.batch_size, self.shuffle, self.collate_fn = dataset, batch_size, shuffle, collate_fn
        self.workers, self.prefetch, self.thread = workers, prefetch, thread
        self._pool = None

    def __len__(self):
        return (len(self.dataset) + self.batch_size - 1) // self.batch_size

    def close(self):
        if self._pool is not None:
            self._pool.terminate()
            self._pool = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _split(self):
        ds = self.dataset
        return hasattr(ds, "host_args") and hasattr(ds, "from_host")

    def _host_items(self, idx):
        ds = self.dataset
        if self.workers > 0:
            if self._pool is None:
                self._pool = multiprocessing.get_context("spawn").Pool(self.workers)
            return self._pool.imap(_host_load_args, [ds.host_args(j) for j in idx], chunksize=1)
        return (ds.load_host(j) for j in idx)

    def _batches(self, idx):
        """Batches built in the calling thread on the current stream, host halves from _host_items."""
        ds = self.dataset
        if not self._split():
            for i in range(0, len(idx), self.batch_size):
                yield self.collate_fn([ds[j] for j in idx[i:i + self.batch_size]])
            return
        host = self._host_items(idx)
        for i in range(0, len(idx), self.batch_size):
            yield self.collate_fn([ds.from_host(next(host)) for _ in range(min(self.batch_size, len(idx) - i))])

    def __iter__(self):
        n = len(self.dataset)
        # torch.utils.data.DataLoader's draws from torch's global generator, in its order: the
        # iterator's worker base seed (drawn even with num_workers=0 and shuffle off), then
        # RandomSampler's seed for a randperm on a private generator.  Python's `random` stream
        # (which the augmentations draw from, dataset.py:204-300) is left untouched, as under the
        # reference's DataLoader.
        torch.empty((), dtype=torch.int64).random_()
        if self.shuffle:
            seed = int(torch.empty((), dtype=torch.int64).random_().item())
            gen = torch.Generator()
            gen.manual_seed(seed)
            idx = torch.randperm(n, generator=gen).tolist()
        else:
            idx = list(range(n))
        if self.prefetch <= 0 or not torch.cuda.is_available():
            yield from self._batches(idx)
            return
        consumer = torch.cuda.current_stream()
        side = torch.cuda.Stream(device=consumer.device)
        src = self._batches(idx)
        if self.thread:
            yield from self._threaded(src, consumer, side)
            return
        ready = deque()

        def build():  # the next batch's device work, enqueued on the side stream
            with torch.cuda.stream(side):
                b = next(src, None)
                if b is None:
                    return False
                ev = torch.cuda.Event()
                ev.record(side)
            ready.append((b, ev))
            return True

        more = True
        while more and len(ready) < self.prefetch:
            more = build()
        while ready:
            b, ev = ready.popleft()
            if more:
                more = build()
            consumer.wait_event(ev)
            _record(b, consumer)
            yield b


    def _threaded(self, src, consumer, side):
        """The device half of every batch built by one producer thread on the side stream, up to
        `prefetch` batches ahead (every Python `random` draw still in item order: one producer).
        Pays off when the consumer's own host work per batch is short -- Trainer.step_graph's single
        graph launch -- so the two threads overlap instead of ping-ponging the GIL."""
        q = queue.Queue(maxsize=self.prefetch)
        stop = threading.Event()

        def put(item):
            while not stop.is_set():
                try:
                    q.put(item, timeout=0.1)
                    return True
                except queue.Full:
                    continue
            return False

        def producer():
            try:
                torch.cuda.set_device(consumer.device)
                with torch.cuda.stream(side):
                    for b in src:
                        ev = torch.cuda.Event()
                        ev.record(side)
                        if not put((b, ev)):
                            return
                put(None)
            except BaseException as e:  # handed to the consumer, raised there
                put(e)

        t = threading.Thread(target=producer, name="eunet-loader", daemon=True)
        t.start()
        try:
            while True:
                item = q.get()
                if item is None:
                    return
                if isinstance(item, BaseException):
                    raise item
                b, ev = item
                consumer.wait_event(ev)
                _record(b, consumer)
                yield b
        finally:
            stop.set()
            t.join()


def _record(obj, stream):
    """record_stream every device tensor of a batch on the consuming stream (the caching allocator
    must not reuse their blocks while that stream still reads them)."""
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            obj.record_stream(stream)
    elif isinstance(obj, dict):
        for v in obj.values():
            _record(v, stream)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _record(v, stream)
