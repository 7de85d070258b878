// imagedec.h — image files for image_texture / map_Kd textures (the reference's imageio::load_image,
// imageio.cpp:11-15 = stbi_load(path, &w, &h, &c, 0) of the vendored stb_image v2.27): JPEG (baseline and progressive,
// Huffman, 8-bit, any integer sampling factors) and PNG (every color type and bit depth, Adam7), decoded to the bytes
// stb_image returns -- native channel count, 8 bits per channel, row 0 = top.  Written from the JPEG (ITU-T T.81) and
// PNG (ISO/IEC 15948) specifications; where the standards leave arithmetic to the decoder (JPEG's inverse DCT,
// YCbCr -> RGB, chroma upsampling, 16 -> 8 bit) the stb_image formulas are restated so the bytes match
// (tests/test_imagedec.py pins them against the reference's own decodes).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace art {

struct DecodedImage {
    int w = 0, h = 0, channels = 0;
    std::vector<uint8_t> data;  // h * w * channels
};

DecodedImage decode_jpeg(const uint8_t* bytes, size_t n);
DecodedImage decode_png(const uint8_t* bytes, size_t n);
// By content (JPEG SOI / PNG signature); throws std::runtime_error with the reason on anything it cannot decode.
DecodedImage decode_image(const uint8_t* bytes, size_t n);
DecodedImage load_image_file(const std::string& path);

}  // namespace art
