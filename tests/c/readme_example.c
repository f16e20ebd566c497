/*
 * readme_example.c -- the reference's README usage example for RS
 * (/root/reference/README.md:63-101: encode a 64-byte message, flip two
 * bytes, decode) written as a drop-in check: it includes only the
 * reference's public header, include/poporon.h, and links against
 * libpoporon_amd.so.  Exit status 0 iff both errors are corrected and the
 * message reads back.
 */
#include <poporon.h>
#include <stdio.h>
#include <string.h>

int main(void)
{
    static const char text[] = "Hello, Reed-Solomon!";
    poporon_config_t *config = poporon_config_rs_default();
    poporon_t *pprn = poporon_create(config);
    uint8_t data[64];
    uint8_t parity[32];
    size_t corrected_num = 0;
    int status = 1;

    if (!pprn) {
        fprintf(stderr, "Failed to create poporon instance\n");
        poporon_config_destroy(config);
        return 1;
    }
    memset(data, 0, sizeof(data));
    memcpy(data, text, sizeof(text) - 1);
    if (!poporon_encode(pprn, data, sizeof(data), parity)) {
        fprintf(stderr, "poporon_encode failed\n");
        goto done;
    }
    data[0] ^= 0xFF; /* two symbol errors */
    data[10] ^= 0xAA;
    if (poporon_decode(pprn, data, sizeof(data), parity, &corrected_num)) {
        printf("Corrected %zu errors\n", corrected_num);
        printf("Decoded: %s\n", (const char *)data);
        status = (corrected_num == 2 && strcmp((const char *)data, text) == 0) ? 0 : 1;
    } else {
        fprintf(stderr, "poporon_decode failed\n");
    }
done:
    poporon_destroy(pprn);
    poporon_config_destroy(config);
    return status;
}
